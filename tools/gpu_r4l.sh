#!/bin/bash
# split histogram entries with b(o_0) loaded ahead of the prologue: parity, then A/B against the old layout
set -uo pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_group.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py tests/test_gpu_peer.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
for r in 1 2 3; do
  for L in libhmmbw_h0.so libhmmbw.so; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
  done
done
# wide kernel, compile-time ablations (release schedule): 0 none, 4 no gamma rows, 8 no alpha_hat traffic, 16 no barrier
echo "== wide own-block-first"
timeout -k 10 200 python -u tools/wide_chunk_times.py --R 4096,6250 --lib $PWD/hmm_training_amd/libhmmbw_own.so > $OUT/wide_own.txt 2>&1 || { tail -20 $OUT/wide_own.txt; exit 1; }
grep -E "====|cycles/step|duration" $OUT/wide_own.txt
timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/bench_cfg5.log 2>&1 || { tail -20 $OUT/bench_cfg5.log; exit 1; }
grep '"metric"' $OUT/bench_cfg5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('cfg5 value %.4g ms/step %.1f us kernel %.1f us estep %.1f us' % (d['value'], d['ms_per_step']*1e3, r['kernel_ms']*1e3, r['bounds']['simd_mfma']['kernel_ms']*1e3))"
for CT in 0 8 16; do
  echo "== wide CT=$CT"
  timeout -k 10 200 python -u tools/wide_chunk_times.py --R 4096,6250 --lib $PWD/hmm_training_amd/libhmmbw_ct$CT.so > $OUT/wide_ct$CT.txt 2>&1 || { tail -20 $OUT/wide_ct$CT.txt; exit 1; }
  grep -E "====|cycles/step|duration" $OUT/wide_ct$CT.txt
done
