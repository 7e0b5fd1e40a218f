#!/bin/bash
# Round 5: isolate the wide peer failure by receive-region memory kind, then the rest of call r5a.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5b
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
for M in coarse finegrained uncached; do
  step peer n64 $M
  HMMBW_PEER_MEM=$M timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
    -k "n64_k1024_tiny" > $O/peer_n64_$M.log 2>&1
  echo "rc=$?"; tail -2 $O/peer_n64_$M.log
done
step rest
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py \
  tests/test_gpu_multirank.py -k "(work_queue or peer) and not n64_k1024_tiny" > $O/pytest_rest.log 2>&1
echo "rc=$?"; tail -3 $O/pytest_rest.log
step phase T8
timeout -k 10 300 python -u tools/phase_times.py --R 1024,8192 --T 8 --iters 6 > $O/phase_T8.log 2>&1 || exit 1
step phase T200
timeout -k 10 300 python -u tools/phase_times.py --R 10000 --T 200 > $O/phase_T200.log 2>&1 || exit 1
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
step done
