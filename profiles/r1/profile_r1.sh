#!/bin/bash
# Profile the headline bench under rocprofv3 (kernel trace + stats, then one PMC pass per counter)
# and the PMC calibration program.  Run on the GPU box from the repo root:
#   bash tools/profile_r1.sh <tag>
set -euo pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o "$OUT/pmc_calib" "$R/tools/pmc_calib.hip"
cd /tmp
BENCH="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/bench_trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- python3 $BENCH > "$OUT/bench_pmc_$C.log" 2>&1
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- "$OUT/pmc_calib" > "$OUT/calib_$C.log" 2>&1
done
echo done
