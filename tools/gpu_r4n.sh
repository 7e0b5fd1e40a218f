#!/bin/bash
# parity with the natural forward + own-first backward; cfg5 line and timeline; then the r4 profiles, part a
set -uo pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_deterministic.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py tests/test_gpu_peer.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/bench_cfg5.log 2>&1 || { tail -20 $OUT/bench_cfg5.log; exit 1; }
grep '"metric"' $OUT/bench_cfg5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('cfg5 value %.4g ms/step %.1f us kernel %.1f us estep %.1f us' % (d['value'], d['ms_per_step']*1e3, r['kernel_ms']*1e3, r['bounds']['simd_mfma']['kernel_ms']*1e3))"
timeout -k 10 200 python -u tools/wide_chunk_times.py --R 4096,6250 --lib $PWD/hmm_training_amd/libhmmbw_own.so > $OUT/wide_own.txt 2>&1 || { tail -20 $OUT/wide_own.txt; exit 1; }
grep -E "====|cycles/step|duration" $OUT/wide_own.txt
bash tools/profile_all.sh r4 a > $OUT/prof_a.log 2>&1 || { tail -20 $OUT/prof_a.log; exit 1; }
tail -3 $OUT/prof_a.log
