#!/bin/bash
# A/B: static wave priority (HMMBW_PRIO 0/1/2) on the small E-step, interleaved rounds; then full-size tests
set -uo pipefail
OUT=gpurun_out/r4f
mkdir -p $OUT
for r in 1 2 3; do
  for P in 0 1 2; do
    echo "== prio $P round $r"
    HMMBW_PRIO=$P timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
    HMMBW_PRIO=$P timeout -k 10 120 python -u tools/occupancy.py --Rs 10000 --ablate 0 --iters 50 --topology dense 2>&1 | grep "R=" || exit 1
  done
done
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread --durations=15 tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|s call|Error" $OUT/pytest.log | tail -40
exit $rc
