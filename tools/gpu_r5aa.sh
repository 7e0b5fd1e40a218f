#!/bin/bash
# Round 5: warm phase timelines of the dense kernel with the split extra waves (and without, HMMBW_SPLIT_EXTRA=0).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 200 python3 tools/phase_times.py --R 10000 --topology dense > $O/phase_dense_split.log 2>&1 || exit 1
HMMBW_SPLIT_EXTRA=0 timeout -k 10 200 python3 tools/phase_times.py --R 10000 --topology dense > $O/phase_dense_nosplit.log 2>&1 || exit 1
grep -v amdgpu $O/phase_dense_split.log $O/phase_dense_nosplit.log
