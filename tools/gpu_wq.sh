#!/bin/bash
# wide work queue: parity (new tests + the full-size wide tests), then cfg5 shard / whole A/B (HMMBW_WIDE_WQ)
set -uo pipefail
OUT=gpurun_out/wq
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "work_queue" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
grep -E "passed|failed" $OUT/t1.log | tail -3
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_fullsize.py -k "cfg5 or wide" > $OUT/t2.log 2>&1 || { tail -40 $OUT/t2.log; exit 1; }
grep -E "passed|failed|PASSED" $OUT/t2.log | tail -12
for r in 1 2; do
  for w in 1 0; do
    HMMBW_WIDE_WQ=$w timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/cfg5_wq$w.$r.json 2> $OUT/cfg5_wq$w.$r.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/cfg5_wq$w.$r.json').read().strip().splitlines()[-1]); print('cfg5 wq=$w', round(d['ms_per_step']*1000,1), 'us/step', d['roofline'].get('kernel_ms'))"
  done
done
for w in 1 0; do
  HMMBW_WIDE_WQ=$w timeout -k 10 300 python -u bench.py --workload cfg5 --R 50000 --steps 3 --warmup 1 --no-cpu-baseline --no-synced > $OUT/cfg5w_wq$w.json 2> $OUT/cfg5w_wq$w.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/cfg5w_wq$w.json').read().strip().splitlines()[-1]); print('cfg5 whole wq=$w', round(d['ms_per_step']*1000,1), 'us/step')"
done
