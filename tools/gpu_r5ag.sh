#!/bin/bash
# Round 5: joined spread map (HMMBW_JOIN=1: the extra workgroups' waves run as waves 4.. of the full workgroups,
# one 8-wave workgroup per CU, k_estep_join) against the release map, left-to-right cfg3; parity first.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5ag
mkdir -p $O
export PYTHONUNBUFFERED=1
HMMBW_JOIN=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "cfg3_full_size_vs_oracle or spread_extra_waves_ragged" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:28s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
for i in 1 2 3; do
  for J in 0 1; do
    HMMBW_JOIN=$J timeout -k 10 200 python -u bench.py --steps 300 --no-cpu-baseline --no-synced > $O/lr_j$J.log 2>&1 || exit 1
    summ $O/lr_j$J.log "lr join=$J"
  done
done
for J in 0 1; do
  HMMBW_JOIN=$J timeout -k 10 200 python -u bench.py --steps 300 --no-cpu-baseline --no-synced --symbols H > $O/lrH_j$J.log 2>&1 || exit 1
  summ $O/lrH_j$J.log "lrH join=$J"
done
echo done
