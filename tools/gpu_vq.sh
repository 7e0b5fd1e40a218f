set -o pipefail
mkdir -p gpurun_out/vq
timeout -k 10 300 python -u -m pytest tests/test_gpu_vq.py -x -v --timeout 120 --timeout-method thread > gpurun_out/vq/tests.log 2>&1 || { tail -40 gpurun_out/vq/tests.log; exit 1; }
tail -2 gpurun_out/vq/tests.log
timeout -k 10 120 python -u tools/bench_vq.py > gpurun_out/vq/vq.log 2>&1 || { tail -20 gpurun_out/vq/vq.log; exit 1; }
grep kernel gpurun_out/vq/vq.log
