#!/bin/bash
# Refresh every profile of one round on the GPU box (run from the repo root):
#   bash tools/profile_all.sh <tag>
# rocprofv3 kernel trace + stats per workload, then one PMC pass per counter for the headline
# (never combined with a trace domain), the PMC calibration program, and the bench JSON lines.
set -uo pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
hipcc --offload-arch=gfx950 -O3 -o "$OUT/pmc_calib" "$R/tools/pmc_calib.hip" || exit 1
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  step calib $C
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- "$OUT/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || exit 1
done
for TOPO in left_to_right dense; do
  BENCH="$R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --topology $TOPO"
  step trace $TOPO
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$TOPO" -o run -- python3 $BENCH > "$OUT/bench_trace_$TOPO.log" 2>&1 || exit 1
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc $C $TOPO
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$TOPO" -o run -- python3 $BENCH > "$OUT/bench_pmc_${C}_$TOPO.log" 2>&1 || exit 1
  done
done
step trace cfg5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_cfg5" -o run -- python3 $R/bench.py --N 64 --K 1024 --T 400 --R 6250 --steps 10 --warmup 2 --topology dense --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || exit 1
step trace cfg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_cfg2" -o run -- python3 $R/tools/bench_cfg2.py --no-cpu > "$OUT/bench_cfg2.log" 2>&1 || exit 1
step trace vq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_vq" -o run -- python3 $R/tools/bench_vq.py > "$OUT/bench_vq.log" 2>&1 || exit 1
step bench
timeout -k 10 300 python3 "$R/bench.py" > "$OUT/bench_full.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --topology dense --no-cpu-baseline > "$OUT/bench_dense.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/tools/bench_cfg2.py" > "$OUT/bench_cfg2_full.log" 2>&1 || exit 1
step done
