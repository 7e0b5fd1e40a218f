#!/bin/bash
# split histogram entries with b(o_0) loaded ahead of the prologue: parity, then A/B against the old layout
set -uo pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_group.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
for r in 1 2 3; do
  for L in libhmmbw_h0.so libhmmbw.so; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
  done
done
# wide kernel, compile-time ablations (release schedule): 0 none, 4 no gamma rows, 8 no alpha_hat traffic, 16 no barrier
for CT in 0 4 8 16; do
  echo "== wide CT=$CT"
  timeout -k 10 200 python -u tools/wide_chunk_times.py --R 4096,6250 --lib $PWD/hmm_training_amd/libhmmbw_ct$CT.so > $OUT/wide_ct$CT.txt 2>&1 || { tail -20 $OUT/wide_ct$CT.txt; exit 1; }
  grep -E "====|cycles/step|duration" $OUT/wide_ct$CT.txt
done
