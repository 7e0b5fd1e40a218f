#!/bin/bash
# Round 5: the wide peer all-reduce test alone, by receive-region memory kind (stop at the first failure).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5c
mkdir -p $O
export PYTHONUNBUFFERED=1
for M in coarse finegrained uncached; do
  echo "[$(date +%T)] $M"
  HMMBW_PEER_MEM=$M timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
    -k "test_peer_allreduce_vs_oracle or native_loop or wait_is_bounded" > $O/peer_$M.log 2>&1
  rc=$?; echo "rc=$rc"; tail -2 $O/peer_$M.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
