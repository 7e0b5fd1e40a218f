#!/bin/bash
# A/B: the dense path's stored z_t with nontemporal stores / loads, cfg3 dense, interleaved
set -uo pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
for r in 1 2 3; do
  for L in libhmmbw.so libhmmbw_nt.so; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py --Rs 10000 --ablate 0 --iters 100 --topology dense 2>&1 | grep "R=" || exit 1
  done
done
