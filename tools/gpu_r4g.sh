#!/bin/bash
# dense table layout: parity of the small-kernel paths, then A/B vs the baseline library (interleaved);
# priority A/B; then the full-size tests
set -uo pipefail
OUT=gpurun_out/r4g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_group.py tests/test_gpu_fuzz.py > $OUT/pytest_small.log 2>&1
rc=$?; tail -3 $OUT/pytest_small.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_small.log | head; exit $rc; fi
for r in 1 2 3; do
  for L in libhmmbw_base.so libhmmbw.so; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 50 --topology dense 2>&1 | grep "R=" || exit 1
  done
  for P in 0 1 2; do
    echo "== prio $P round $r"
    HMMBW_PRIO=$P timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
  done
done
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread --durations=15 tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|s call|Error" $OUT/pytest.log | tail -40
exit $rc
