#!/bin/bash
# A/B: work-queue hand-off through agent-scope stores / loads (libhmmbw_wt.so) against release / acquire fences
set -uo pipefail
OUT=gpurun_out/wqwt
mkdir -p $OUT
WT=$PWD/hmm_training_amd/libhmmbw_wt.so
HMMBW_LIB=$WT timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "work_queue" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
grep -E "passed|failed" $OUT/t.log | tail -2
for r in 1 2; do
  for L in libhmmbw.so libhmmbw_wt.so; do
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 300 python -u bench.py --workload cfg5 --R 50000 --steps 3 --warmup 1 --no-cpu-baseline --no-synced > $OUT/w_$L.$r.json 2> $OUT/w_$L.$r.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/w_$L.$r.json').read().strip().splitlines()[-1]); print('whole $L', round(d['ms_per_step']*1000,1))"
    HMMBW_WIDE_WQ=1 HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/s_$L.$r.json 2> $OUT/s_$L.$r.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/s_$L.$r.json').read().strip().splitlines()[-1]); print('shard wq=1 $L', round(d['ms_per_step']*1000,1))"
  done
done
