#!/bin/bash
# parity with the own-block-first wide exchange; cfg5 and cfg3 bench lines; wide timeline old vs new
set -uo pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_group.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py tests/test_gpu_peer.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/bench_cfg5_$r.log 2>&1 || { tail -20 $OUT/bench_cfg5_$r.log; exit 1; }
  grep '"metric"' $OUT/bench_cfg5_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('cfg5 value %.4g ms/step %.1f us kernel %.1f us estep %.1f us' % (d['value'], d['ms_per_step']*1e3, r['kernel_ms']*1e3, r['bounds']['simd_mfma']['kernel_ms']*1e3))"
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-synced > $OUT/bench_lr.log 2>&1 || { tail -20 $OUT/bench_lr.log; exit 1; }
grep '"metric"' $OUT/bench_lr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lr value %.4g ms/step %.2f us kernel %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))"
for L in ct0 own; do
  echo "== wide $L"
  timeout -k 10 200 python -u tools/wide_chunk_times.py --R 4096,6250 --lib $PWD/hmm_training_amd/libhmmbw_$L.so > $OUT/wide_$L.txt 2>&1 || { tail -20 $OUT/wide_$L.txt; exit 1; }
  grep -E "====|cycles/step|duration" $OUT/wide_$L.txt
done
