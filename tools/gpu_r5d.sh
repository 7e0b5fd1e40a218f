#!/bin/bash
# Round 5: fixed-cost ablations (steady state), the half-length extra-wave bound, peer/WQ tests, bench line.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5d
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
L=$R/hmm_training_amd
step ablate
for lib in libhmmbw.so libhmmbw_xhalf.so; do
  HMMBW_LIB=$L/$lib timeout -k 10 200 python -u tools/steady_ablate.py --R 10000 --T 200 >> $O/ablate.log 2>&1 || exit 1
done
HMMBW_LIB=$L/libhmmbw.so timeout -k 10 200 python -u tools/steady_ablate.py --R 8192 --T 8 >> $O/ablate.log 2>&1 || exit 1
HMMBW_LIB=$L/libhmmbw.so timeout -k 10 200 python -u tools/steady_ablate.py --R 1024 --T 8 >> $O/ablate.log 2>&1 || exit 1
cat $O/ablate.log | grep us/iter
step pytest
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_peer.py tests/test_gpu_multirank.py tests/test_gpu_comm.py \
  -k "work_queue or peer or multirank or comm" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
step done
