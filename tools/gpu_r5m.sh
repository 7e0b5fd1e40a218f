#!/bin/bash
# Round 5: split extra waves (dense only) parity, then the A/B against the previous library (libhmmbw_head.so)
# and split off (HMMBW_SPLIT_EXTRA=0), alternating on one box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5m
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
step parity
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "split_extra or spread_extra or cfg3_full_size" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
  for V in head new new_s0; do
    L=libhmmbw.so; E=""
    [ $V = head ] && L=libhmmbw_head.so
    [ $V = new_s0 ] && E="HMMBW_SPLIT_EXTRA=0"
    for TOPO in left_to_right dense; do
      env $E HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 200 --topology $TOPO --no-cpu-baseline --no-synced > $O/${V}_$TOPO.log 2>&1 || exit 1
      summ $O/${V}_$TOPO.log "$V $TOPO"
    done
  done
done
step done
