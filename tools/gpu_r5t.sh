#!/bin/bash
# Round 5 diagnostics: the extra workgroups without their statistics flush (libhmmbw_xnf.so, results wrong):
# the most that merging the extra groups into the full workgroups' flush could gain.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for L in libhmmbw.so libhmmbw_xnf.so libhmmbw.so libhmmbw_xnf.so; do
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged 2>&1 | grep merged
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged --topology dense 2>&1 | grep merged
done
