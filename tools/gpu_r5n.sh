#!/bin/bash
# Round 5: split extra waves in the left-to-right kernel (libhmmbw_splr.so, -DHMMBW_SPLIT_LR=1) against the
# release (no split for left-to-right): parity, then cfg3 LR / LR-H alternating.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5n
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
HMMBW_LIB=$R/hmm_training_amd/libhmmbw_splr.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "split_extra or spread_extra or cfg3_full_size" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
  for V in rel splr splr_s0; do
    L=libhmmbw.so; E=""
    [ $V != rel ] && L=libhmmbw_splr.so
    [ $V = splr_s0 ] && E="HMMBW_SPLIT_EXTRA=0"
    env $E HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-synced > $O/${V}_lr.log 2>&1 || exit 1
    summ $O/${V}_lr.log "$V lr"
  done
done
step done
