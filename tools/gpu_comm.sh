set -o pipefail
mkdir -p gpurun_out/comm
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/comm/tests.log 2>&1 || { tail -40 gpurun_out/comm/tests.log; exit 1; }
tail -2 gpurun_out/comm/tests.log
timeout -k 10 300 python -u tools/multirank_overhead.py > gpurun_out/comm/mr.log 2>&1 || { tail -30 gpurun_out/comm/mr.log; exit 1; }
tail -1 gpurun_out/comm/mr.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/comm/all.log 2>&1 || { tail -30 gpurun_out/comm/all.log; exit 1; }
tail -2 gpurun_out/comm/all.log
