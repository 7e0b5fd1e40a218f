#!/bin/bash
# Round 5: LR E-step at warm clocks over R (occupancy curve) and over T at R = 10,000 (per-step slope and the
# T-independent intercept: the fixed cost per launch), bench.py --R/--T, 200 steps each.
set -uo pipefail
R0=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R0"
O=gpurun_out/r5ac
mkdir -p $O
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:16s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={r.get('launch_map',{}).get('workgroups')}/{r.get('launch_map',{}).get('extra_waves')}")
PY
}
for R in 1024 4096 8192 9000 10000 11000 12500 16384; do
  timeout -k 10 200 python -u bench.py --R $R --steps 200 --no-cpu-baseline --no-synced > $O/r.log 2>&1 || exit 1
  summ $O/r.log "R=$R T=200"
done
for T in 8 25 50 100 200 400; do
  timeout -k 10 200 python -u bench.py --T $T --steps 200 --no-cpu-baseline --no-synced > $O/t.log 2>&1 || exit 1
  summ $O/t.log "R=10000 T=$T"
done
for T in 8 50 200; do
  timeout -k 10 200 python -u bench.py --R 8192 --T $T --steps 200 --no-cpu-baseline --no-synced > $O/t.log 2>&1 || exit 1
  summ $O/t.log "R=8192 T=$T"
done
