#!/bin/bash
# Copy the summaries of one tools/profile_all.sh run (gpurun_out/prof_<tag>) into profiles/<dest>/ and
# rebuild the per-launch traffic JSONs bench.py reads.   bash tools/collect_profiles.sh <tag> <dest>
set -euo pipefail
TAG=$1; DEST=$2
SRC=gpurun_out/prof_$TAG
mkdir -p "profiles/$DEST"
export HMMBW_PROFILE_SHA=$(cat "$SRC/kernel_src_sha16.txt" 2>/dev/null || true)
export HMMBW_PROFILE_UTC=$(cat "$SRC/collected_utc.txt" 2>/dev/null || true)
cp "$SRC/calib_FETCH_SIZE/run_counter_collection.csv" "profiles/$DEST/pmc_calib_FETCH_SIZE.csv"
cp "$SRC/calib_WRITE_SIZE/run_counter_collection.csv" "profiles/$DEST/pmc_calib_WRITE_SIZE.csv"
declare -A KEY=([lr_cfg3]=R10000_T200_N8_K256_left_to_right [lrH_cfg3]=R10000_T200_N8_K256_left_to_right_H
                [dense_cfg3]=R10000_T200_N8_K256_dense [cfg5]=R6250_T400_N64_K1024_dense
                [cfg4shard]=R12500_T200_N8_K256_left_to_right)
declare -A KER=([lr_cfg3]=k_estep_join [lrH_cfg3]=k_estep_join [dense_cfg3]=k_estep_join
                [cfg5]="k_estep_mfma,k_bnum_gather" [cfg4shard]=k_estep_join)
for W in lr_cfg3 lrH_cfg3 dense_cfg3 cfg5 cfg4shard; do
  [ -d "$SRC/trace_$W" ] || { echo "skip $W (not in this run)"; continue; }
  cp "$SRC/trace_$W/run_kernel_stats.csv" "profiles/$DEST/kernel_stats_$W.csv"
  for C in FETCH_SIZE WRITE_SIZE SQ SQ2; do
    cp "$SRC/pmc_${C}_$W/run_counter_collection.csv" "profiles/$DEST/pmc_${C}_$W.csv"
  done
  python3 tools/traffic_summary.py --fetch "profiles/$DEST/pmc_FETCH_SIZE_$W.csv" \
    --write "profiles/$DEST/pmc_WRITE_SIZE_$W.csv" \
    --calib-fetch "profiles/$DEST/pmc_calib_FETCH_SIZE.csv" --calib-write "profiles/$DEST/pmc_calib_WRITE_SIZE.csv" \
    --kernel "${KER[$W]}" --config-key "${KEY[$W]}" --out "profiles/$DEST/traffic_$W.json"
  python3 tools/pmc_summary.py "profiles/$DEST/pmc_SQ_$W.csv,profiles/$DEST/pmc_SQ2_$W.csv" "${KER[$W]}" --config-key "${KEY[$W]}" \
    --kernel-stats "profiles/$DEST/kernel_stats_$W.csv" > "profiles/$DEST/sq_$W.json"
done
for W in cfg2 vq; do
  [ -d "$SRC/trace_$W" ] && cp "$SRC/trace_$W/run_kernel_stats.csv" "profiles/$DEST/kernel_stats_$W.csv"
done
[ -f "$SRC/bench_full.log" ] || exit 0  # part a: no bench lines
grep -h '"metric"' "$SRC/bench_full.log" > "profiles/$DEST/bench_lr_cfg3.json"
grep -h '"metric"' "$SRC/bench_dense.log" > "profiles/$DEST/bench_dense_cfg3.json"
grep -h '"metric"' "$SRC/bench_H.log" > "profiles/$DEST/bench_lrH_cfg3.json"
grep -h '"metric"' "$SRC/bench_cfg5.log" > "profiles/$DEST/bench_cfg5.json"
grep -h '"metric"' "$SRC/bench_cfg4shard.log" > "profiles/$DEST/bench_cfg4shard.json"
grep -h '"metric"' "$SRC/bench_cfg5_50k.log" > "profiles/$DEST/bench_cfg5_50k.json"
grep -h '"workload"' "$SRC/bench_cfg2_full.log" > "profiles/$DEST/bench_cfg2_grouped.json"
grep -h '"kernel"' "$SRC/bench_vq.log" > "profiles/$DEST/bench_vq.json"
