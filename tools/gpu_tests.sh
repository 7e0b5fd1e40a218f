#!/bin/bash
# One GPU call: the given pytest selection (default: the whole -m gpu suite), then optional bench args.
#   bash tools/gpu_tests.sh <tag> [pytest -k expression]
set -uo pipefail
TAG=${1:-tests}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${SEL[@]}" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.log"
exit $rc
