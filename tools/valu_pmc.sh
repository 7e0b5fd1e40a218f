#!/bin/bash
set -uo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/valu
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for T in 100 200 400; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/T$T -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-synced --T $T > $OUT/T$T.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py $OUT/T$T/run_counter_collection.csv k_estep_small > $OUT/T$T.json || exit 1
done
cat $OUT/T*.json
