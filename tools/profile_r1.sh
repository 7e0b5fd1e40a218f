#!/bin/bash
# Profile the headline bench under rocprofv3 (kernel trace + stats, then one PMC pass per counter,
# never combined with a trace domain) for each topology, plus the PMC calibration program.
# Run on the GPU box from the repo root:   bash tools/profile_r1.sh <tag>
set -euo pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o "$OUT/pmc_calib" "$R/tools/pmc_calib.hip"
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- "$OUT/pmc_calib" > "$OUT/calib_$C.log" 2>&1
done
for TOPO in left_to_right dense; do
  BENCH="$R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --topology $TOPO"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$TOPO" -o run -- python3 $BENCH > "$OUT/bench_trace_$TOPO.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$TOPO" -o run -- python3 $BENCH > "$OUT/bench_pmc_${C}_$TOPO.log" 2>&1
  done
done
timeout -k 10 300 python3 "$R/bench.py" > "$OUT/bench_full.log" 2>&1
timeout -k 10 300 python3 "$R/bench.py" --topology dense --no-cpu-baseline > "$OUT/bench_dense.log" 2>&1
echo done
