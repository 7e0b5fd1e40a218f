#!/bin/bash
# wide chunk timeline (one vs two tiles per CU), LR bench with the extra-wave priority default, LR SQ counters
set -uo pipefail
OUT=gpurun_out/r4j
mkdir -p $OUT
timeout -k 10 300 python -u tools/wide_chunk_times.py --R 4096,6250 > $OUT/wide_chunks.txt 2>&1 || { tail -20 $OUT/wide_chunks.txt; exit 1; }
cat $OUT/wide_chunks.txt
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lr value %.4g ms/step %.2f us kernel %.2f us synced %.2f us dropin %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['synced']['median_ms_per_iter_with_d2h']*1e3, d['synced']['dropin_train_ms_per_iter']*1e3))"
bash tools/lr_pmc.sh > $OUT/lr_pmc.txt 2>&1 || { tail -30 $OUT/lr_pmc.txt; exit 1; }
grep -E "==|ACTIVE|WAIT|LEVEL|BUSY|WAVE_CYCLES|SQ_WAVES|IDX|CONFLICT|GRBM" $OUT/lr_pmc.txt
