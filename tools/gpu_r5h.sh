#!/bin/bash
# Round 5: LR prologue A/B (statistics loads before the zero-clearing stores, no padding loads):
# release libhmmbw.so against libhmmbw_pro.so, steady-state at cfg3 and T = 8, then the bench line.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5h
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
for L in libhmmbw.so libhmmbw_pro.so libhmmbw.so libhmmbw_pro.so; do
  step steady $L
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged >> $O/steady.log 2>&1 || exit 1
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged --R 8192 --T 8 >> $O/steady.log 2>&1 || exit 1
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged --topology dense >> $O/steady.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/steady.log
step done
