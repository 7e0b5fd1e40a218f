#!/bin/bash
# Round 5: the bench lines again, after the refreshed profiles are in the tree (so every bound's provenance is fresh).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5v
mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.log 2>&1 || exit 1; }
run lr_cfg3
run dense_cfg3 --topology dense --no-cpu-baseline
run lrH_cfg3 --symbols H --no-cpu-baseline
run cfg4shard --workload cfg4 --no-cpu-baseline
run cfg5 --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline
run cfg5_50k --workload cfg5 --R 50000 --steps 5 --warmup 1 --no-cpu-baseline --no-synced
echo done
