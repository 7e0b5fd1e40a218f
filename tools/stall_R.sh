#!/bin/bash
# Wave-state and LDS counters of the small E-step at several sequence counts (one rocprofv3 pass per
# counter set, never combined with a trace).   bash tools/stall_R.sh <tag> <lib> "<R list>"
set -uo pipefail
TAG=$1; LIB=$2; RS=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HMMBW_LIB=$R/hmm_training_amd/$LIB
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for RR in $RS; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/R${RR}_p$i" -o run -- python3 "$R/bench.py" --R $RR --steps 10 --warmup 2 --no-cpu-baseline --no-synced --no-kernel-timing > "$OUT/R${RR}_p$i.log" 2>&1 || exit 1
  done
  echo "== R=$RR"
  python3 "$R/tools/pmc_summary.py" "$OUT/R${RR}_p1/run_counter_collection.csv" k_estep | grep -v dispatches
  python3 "$R/tools/pmc_summary.py" "$OUT/R${RR}_p2/run_counter_collection.csv" k_estep | grep -v dispatches
done
