#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread --durations=15 tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|s call|Error" $OUT/pytest.log | tail -40
exit $rc
