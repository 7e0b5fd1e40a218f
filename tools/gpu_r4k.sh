#!/bin/bash
# parity of the split histogram entries (+ b(o_0) from the statistics) and the sorted-row gather; A/B of the
# histogram layout (HMMBW_HIST_SPLIT=0 library) at cfg3 LR / dense and the cfg4 shard, interleaved
set -uo pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_group.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py tests/test_gpu_comm.py tests/test_gpu_status.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
for r in 1 2 3; do
  for L in libhmmbw_h0.so libhmmbw.so; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000 --ablate 0 --iters 50 --topology dense 2>&1 | grep "R=" || exit 1
  done
done
timeout -k 10 400 python -u tools/wide_chunk_times.py --R 4096 --ablate 0,16,8,24,28 > $OUT/wide_abl.txt 2>&1 || { tail -20 $OUT/wide_abl.txt; exit 1; }
grep -E "====|cycles/step|duration" $OUT/wide_abl.txt
