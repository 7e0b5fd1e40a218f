#!/bin/bash
# the work-queue and full-size wide parity tests on the release library, then the whole-cfg5 bench line
set -uo pipefail
OUT=gpurun_out/wqf
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -k "work_queue or cfg5 or wide" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
grep -E "passed|failed" $OUT/t.log | tail -2
timeout -k 10 300 python -u bench.py --workload cfg5 --R 50000 --steps 3 --warmup 1 --no-cpu-baseline --no-synced > $OUT/whole.json 2> $OUT/whole.err || exit 1
tail -1 $OUT/whole.json | cut -c1-220
