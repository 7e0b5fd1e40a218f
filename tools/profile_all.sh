#!/bin/bash
# Refresh every profile of one round on the GPU box (run from the repo root):
#   bash tools/profile_all.sh <tag> [part]
# part: all (default), a (calibration + the cfg3 workloads) or b (cfg5, cfg4 shard, cfg2, vq, bench lines):
# the halves fit one gpurun call each
# rocprofv3 kernel trace + stats per workload, then separate PMC passes (never combined with a
# trace domain): FETCH_SIZE, WRITE_SIZE (HBM traffic, corrected by the tools/pmc_calib.hip run) and an
# SQ/LDS pass (bank conflicts, VALU/LDS instruction counts), plus the bench JSON lines.
set -uo pipefail
TAG=${1:-r2}
PART=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
# provenance of every summary made from this run (tools/collect_profiles.sh stamps them)
(cd "$R" && python3 -c "import bench; print(bench.kernel_source_hash())") > "$OUT/kernel_src_sha16.txt"
date -u +%Y-%m-%dT%H:%M:%SZ > "$OUT/collected_utc.txt"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
cd /tmp
WLS="lr_cfg3 lrH_cfg3 dense_cfg3 cfg5 cfg4shard"
[ "$PART" = a ] && WLS="lr_cfg3 lrH_cfg3 dense_cfg3"
[ "$PART" = b ] && WLS="cfg5 cfg4shard"
if [ "$PART" != b ]; then
hipcc --offload-arch=gfx950 -O3 -o "$OUT/pmc_calib" "$R/tools/pmc_calib.hip" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  step calib $C
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- "$OUT/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || exit 1
done
fi
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
# instruction mix: fp64 VALU issues over 4 cycles on a SIMD-32, the rest over 2 (MI355X_MICROARCH.md); fp64 MFMA busy
SQ2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES"
declare -A ARGS=(
  [lr_cfg3]="--steps 20 --warmup 3 --no-cpu-baseline --no-synced"
  [lrH_cfg3]="--steps 20 --warmup 3 --no-cpu-baseline --no-synced --symbols H"
  [dense_cfg3]="--steps 20 --warmup 3 --no-cpu-baseline --no-synced --topology dense"
  [cfg5]="--steps 5 --warmup 2 --no-cpu-baseline --no-synced --workload cfg5"
  [cfg4shard]="--steps 20 --warmup 3 --no-cpu-baseline --no-synced --workload cfg4"
)
for W in $WLS; do
  BENCH="$R/bench.py ${ARGS[$W]}"
  step trace $W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$W" -o run -- python3 $BENCH > "$OUT/bench_trace_$W.log" 2>&1 || exit 1
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc $C $W
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$W" -o run -- python3 $BENCH > "$OUT/bench_pmc_${C}_$W.log" 2>&1 || exit 1
  done
  step pmc SQ $W
  timeout -k 10 300 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/pmc_SQ_$W" -o run -- python3 $BENCH > "$OUT/bench_pmc_SQ_$W.log" 2>&1 || exit 1
  step pmc SQ2 $W
  timeout -k 10 300 rocprofv3 --pmc $SQ2 --output-format csv -d "$OUT/pmc_SQ2_$W" -o run -- python3 $BENCH > "$OUT/bench_pmc_SQ2_$W.log" 2>&1 || exit 1
done
[ "$PART" = a ] && { step done; exit 0; }
step trace cfg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_cfg2" -o run -- python3 $R/tools/bench_cfg2.py --no-cpu > "$OUT/bench_cfg2.log" 2>&1 || exit 1
step trace vq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_vq" -o run -- python3 $R/tools/bench_vq.py > "$OUT/bench_vq.log" 2>&1 || exit 1
step bench
timeout -k 10 300 python3 "$R/bench.py" > "$OUT/bench_full.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --topology dense --no-cpu-baseline > "$OUT/bench_dense.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --symbols H --no-cpu-baseline > "$OUT/bench_H.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --workload cfg4 --no-cpu-baseline > "$OUT/bench_cfg4shard.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --workload cfg5 --R 50000 --steps 5 --warmup 1 --no-cpu-baseline --no-synced > "$OUT/bench_cfg5_50k.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/tools/bench_cfg2.py" > "$OUT/bench_cfg2_full.log" 2>&1 || exit 1
step done
