#!/bin/bash
# Round 5: the A/B switches read before the spread map (HMMBW_SPLIT_EXTRA=0 gives the xact-2 dense map).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5w
mkdir -p $O
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:20s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={r.get('launch_map',{}).get('workgroups')}/{r.get('launch_map',{}).get('extra_waves')}")
PY
}
timeout -k 10 200 python -u bench.py --topology dense --no-cpu-baseline --no-synced > $O/d.log 2>&1 || exit 1
summ $O/d.log "dense default"
HMMBW_SPLIT_EXTRA=0 timeout -k 10 200 python -u bench.py --topology dense --no-cpu-baseline --no-synced > $O/d0.log 2>&1 || exit 1
summ $O/d0.log "dense split=0"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  -k "split_extra or spread_extra" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
