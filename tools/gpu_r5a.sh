#!/bin/bash
# Round 5, first GPU call: the work-queue / peer tests, the LR fixed-cost phase timeline, a bench line.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5a
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_peer.py tests/test_gpu_multirank.py \
  -k "work_queue or peer or cfg5_shard_is_not" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step phase T8
timeout -k 10 300 python -u tools/phase_times.py --R 1024,8192 --T 8 --iters 6 > $O/phase_T8.log 2>&1 || exit 1
step phase T200
timeout -k 10 300 python -u tools/phase_times.py --R 10000 --T 200 > $O/phase_T200.log 2>&1 || exit 1
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
step done
