#!/bin/bash
# Round 5: cfg4 shard (12,500 sequences, 539 extra waves) with the spread map at xact 3 (HMMBW_XACT=3) against
# full workgroups (the default above 2 extra waves per CU), warm clocks, alternating.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5u
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
  for X in 4 3; do
    for P in 2 0; do
      HMMBW_XACT=$X HMMBW_PRIO=$P timeout -k 10 200 python -u bench.py --workload cfg4 --steps 300 --no-cpu-baseline --no-synced > $O/x$X.log 2>&1 || exit 1
      summ $O/x$X.log "cfg4 xact=$X prio=$P"
    done
  done
done
