#!/bin/bash
# Round 5: the timed region's fixed cost with bench.py's symbols and leg (tools/sync_latency.py), the first
# region of a process, and GPU idle gaps before the region.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/sync_latency.py --bench-params --leg --reps 10 > $O/sync.log 2>&1 || exit 1
for I in 1 10 100; do
  timeout -k 10 120 python -u tools/sync_latency.py --bench-params --leg --reps 6 --idle-ms $I >> $O/sync.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/sync.log
