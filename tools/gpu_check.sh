#!/bin/bash
# One GPU call: parity tests, then the headline bench, dense and cfg5 bench lines.
#   bash tools/gpu_check.sh <tag>
set -uo pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench_lr.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench_lr.log"; exit 1; }
tail -1 "$OUT/bench_lr.log"
timeout -k 10 300 python -u bench.py --topology dense --no-cpu-baseline > "$OUT/bench_dense.log" 2>&1 || { echo "bench dense failed"; tail -30 "$OUT/bench_dense.log"; exit 1; }
tail -1 "$OUT/bench_dense.log"
timeout -k 10 300 python -u bench.py --N 64 --K 1024 --T 400 --R 6250 --steps 10 --warmup 2 --topology dense --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || { echo "bench cfg5 failed"; tail -30 "$OUT/bench_cfg5.log"; exit 1; }
tail -1 "$OUT/bench_cfg5.log"
