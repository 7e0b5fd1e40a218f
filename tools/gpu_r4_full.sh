#!/bin/bash
# the whole GPU suite (as the driver runs it), slowest tests listed
set -uo pipefail
OUT=gpurun_out/r4full
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 > $OUT/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|s call" $OUT/pytest.log | tail -40
exit $rc
