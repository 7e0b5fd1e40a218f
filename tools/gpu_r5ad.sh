#!/bin/bash
# Round 5: warm phase timelines of the LR kernel with the split compiled in (libhmmbw_phsp.so, priority 0, xact 2)
# and of the release (libhmmbw_phase.so, priority 2): where the split's expected gain goes.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5ad
mkdir -p $O
HMMBW_PRIO=0 timeout -k 10 200 python3 tools/phase_times.py --R 10000 --lib $R/hmm_training_amd/libhmmbw_phsp.so > $O/phase_lr_split.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/phase_times.py --R 10000 --lib $R/hmm_training_amd/libhmmbw_phase.so > $O/phase_lr.log 2>&1 || exit 1
grep -v amdgpu $O/phase_lr_split.log $O/phase_lr.log | sed 's#gpurun_out/r5ad/##'
