#!/bin/bash
# Wave-state breakdown of one bench workload's E-step (two SQ passes, never combined with a trace):
#   bash tools/pmc_stall.sh <tag> [bench args]
set -uo pipefail
TAG=${1:-stall}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_LEVEL_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-synced "$@" > "$OUT/p$i.log" 2>&1 || exit 1
done
python3 "$R/tools/pmc_summary.py" "$OUT/p1/run_counter_collection.csv" k_estep > "$OUT/p1.json"
python3 "$R/tools/pmc_summary.py" "$OUT/p2/run_counter_collection.csv" k_estep > "$OUT/p2.json"
cat "$OUT/p1.json" "$OUT/p2.json"
