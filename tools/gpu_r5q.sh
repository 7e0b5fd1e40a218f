#!/bin/bash
# Round 5: the spread map's knobs re-measured at warm clocks: wave priority (HMMBW_PRIO 0/1/2) and active waves
# per extra workgroup (HMMBW_XACT 1/2/3), cfg3 left-to-right and dense (split on), 200 steps each.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5q
mkdir -p $O
export PYTHONUNBUFFERED=1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:28s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={r.get('launch_map',{}).get('workgroups')}/{r.get('launch_map',{}).get('extra_waves')}")
PY
}
for TOPO in left_to_right dense; do
  for P in 2 0 1; do
    for X in 2 1 3; do
      HMMBW_PRIO=$P HMMBW_XACT=$X timeout -k 10 200 python -u bench.py --steps 200 --topology $TOPO --no-cpu-baseline --no-synced > $O/${TOPO}_p${P}_x$X.log 2>&1 || exit 1
      summ $O/${TOPO}_p${P}_x$X.log "$TOPO prio=$P xact=$X"
    done
  done
  HMMBW_PRIO=2 HMMBW_XACT=2 timeout -k 10 200 python -u bench.py --steps 200 --topology $TOPO --no-cpu-baseline --no-synced > $O/${TOPO}_again.log 2>&1 || exit 1
  summ $O/${TOPO}_again.log "$TOPO prio=2 xact=2 again"
done
