#!/bin/bash
# SQ counters of the LR E-step at one and two waves per SIMD (R = 8,192 / 16,384, T = 200): where the
# second wave's time goes (VALU / LDS / waits).   bash tools/lr_pmc.sh   -> gpurun_out/lrpmc/
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lrpmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY"
PB="SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for NR in 8192 16384; do
  for P in PA PB; do
    timeout -s KILL 120 rocprofv3 --pmc ${!P} --output-format csv -d "$OUT/${P}_$NR" -o run -- python3 "$R/tools/occupancy.py" --Rs $NR --T 200 --ablate 0 --iters 20 > "$OUT/log_${P}_$NR.txt" 2>&1 || exit 1
  done
  python3 "$R/tools/pmc_summary.py" "$OUT/PA_$NR/run_counter_collection.csv,$OUT/PB_$NR/run_counter_collection.csv" k_estep_small > "$OUT/sq_$NR.json" || exit 1
  echo "== R=$NR"; cat "$OUT/sq_$NR.json"
done
