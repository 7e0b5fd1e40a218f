set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread > gpurun_out/g2/tests.log 2>&1 || { tail -40 gpurun_out/g2/tests.log; exit 1; }
tail -3 gpurun_out/g2/tests.log
timeout -k 10 120 python -u tools/bench_vq.py > gpurun_out/g2/vq.log 2>&1 || { tail -20 gpurun_out/g2/vq.log; exit 1; }
cat gpurun_out/g2/vq.log
timeout -k 10 300 python -u tools/bench_cfg2.py > gpurun_out/g2/cfg2.log 2>&1 || { tail -20 gpurun_out/g2/cfg2.log; exit 1; }
cat gpurun_out/g2/cfg2.log
