#!/bin/bash
# Copy the summaries of one tools/profile_all.sh run (gpurun_out/prof_<tag>) into profiles/<dest>/ and
# rebuild the per-launch traffic JSONs bench.py reads.   bash tools/collect_profiles.sh <tag> <dest>
set -euo pipefail
TAG=$1; DEST=$2
SRC=gpurun_out/prof_$TAG
mkdir -p "profiles/$DEST"
cp "$SRC/calib_FETCH_SIZE/run_counter_collection.csv" "profiles/$DEST/pmc_calib_FETCH_SIZE.csv"
cp "$SRC/calib_WRITE_SIZE/run_counter_collection.csv" "profiles/$DEST/pmc_calib_WRITE_SIZE.csv"
for TOPO in left_to_right dense; do
  cp "$SRC/trace_$TOPO/run_kernel_stats.csv" "profiles/$DEST/kernel_stats_${TOPO}_cfg3.csv"
  for C in FETCH_SIZE WRITE_SIZE; do
    cp "$SRC/pmc_${C}_$TOPO/run_counter_collection.csv" "profiles/$DEST/pmc_${C}_${TOPO}_cfg3.csv"
  done
  python3 tools/traffic_summary.py --fetch "profiles/$DEST/pmc_FETCH_SIZE_${TOPO}_cfg3.csv" \
    --write "profiles/$DEST/pmc_WRITE_SIZE_${TOPO}_cfg3.csv" \
    --calib-fetch "profiles/$DEST/pmc_calib_FETCH_SIZE.csv" --calib-write "profiles/$DEST/pmc_calib_WRITE_SIZE.csv" \
    --kernel k_estep_small --config-key "R10000_T200_N8_K256_$TOPO" --out "profiles/$DEST/traffic_${TOPO}_cfg3.json"
done
for W in cfg5 cfg2 vq; do
  cp "$SRC/trace_$W/run_kernel_stats.csv" "profiles/$DEST/kernel_stats_$W.csv"
done
grep -h '"metric"' "$SRC/bench_full.log" > "profiles/$DEST/bench_lr_cfg3.json"
grep -h '"metric"' "$SRC/bench_dense.log" > "profiles/$DEST/bench_dense_cfg3.json"
grep -h '"metric"' "$SRC/bench_cfg5.log" > "profiles/$DEST/bench_cfg5.json"
grep -h '"workload"' "$SRC/bench_cfg2_full.log" > "profiles/$DEST/bench_cfg2_grouped.json"
grep -h '"kernel"' "$SRC/bench_vq.log" > "profiles/$DEST/bench_vq.json"
