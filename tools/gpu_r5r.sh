#!/bin/bash
# Round 5: dense defaults (xact 1, priority 0) against the previous ones (HMMBW_XACT=2 HMMBW_PRIO=2), alternating.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5r
mkdir -p $O
export PYTHONUNBUFFERED=1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:20s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={r.get('launch_map',{}).get('workgroups')}/{r.get('launch_map',{}).get('extra_waves')}")
PY
}
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 400 --topology dense --no-cpu-baseline --no-synced > $O/new.log 2>&1 || exit 1
  summ $O/new.log "dense new"
  HMMBW_XACT=2 HMMBW_PRIO=2 timeout -k 10 200 python -u bench.py --steps 400 --topology dense --no-cpu-baseline --no-synced > $O/old.log 2>&1 || exit 1
  summ $O/old.log "dense x2 p2"
  HMMBW_XACT=1 HMMBW_PRIO=0 timeout -k 10 200 python -u bench.py --steps 400 --topology dense --no-cpu-baseline --no-synced > $O/env.log 2>&1 || exit 1
  summ $O/env.log "dense x1 p0 (env)"
done
