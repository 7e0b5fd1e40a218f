#!/bin/bash
# The bench JSON lines of one round's profiles (run on the GPU box after collect_profiles.sh has
# committed the round's traffic / SQ summaries, which bench.py reads):   bash tools/bench_lines.sh <tag>
set -uo pipefail
TAG=${1:-r3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/bench_$TAG
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python3 "$R/bench.py" "$@" > "$OUT/$name.log" 2>&1 || exit 1; }
run lr_cfg3
run dense_cfg3 --topology dense --no-cpu-baseline
run lrH_cfg3 --symbols H --no-cpu-baseline
run cfg4shard --workload cfg4 --no-cpu-baseline
run cfg5 --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline
run cfg5_50k --workload cfg5 --R 50000 --steps 5 --warmup 1 --no-cpu-baseline --no-synced
echo done
