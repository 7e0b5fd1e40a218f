set -o pipefail
mkdir -p gpurun_out/wide
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "wide or n64 or 64 or dense_n16 or safe" --timeout 120 --timeout-method thread > gpurun_out/wide/tests.log 2>&1 || { tail -30 gpurun_out/wide/tests.log; exit 1; }
tail -1 gpurun_out/wide/tests.log
timeout -k 10 300 python -u bench.py --N 64 --K 1024 --T 400 --R 6250 --steps 10 --warmup 2 --topology dense --no-cpu-baseline > gpurun_out/wide/cfg5.log 2>&1 || { tail -20 gpurun_out/wide/cfg5.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"loglik_last": [-0-9.]*' gpurun_out/wide/cfg5.log
