#!/bin/bash
# On-box A/B of library variants with the occupancy timer, interleaved rounds (same box, same clocks).
#   bash tools/ab.sh "<lib1> <lib2> ..." "<occupancy args>" [rounds]
set -uo pipefail
LIBS=$1; ARGS=$2; ROUNDS=${3:-2}
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for L in $LIBS; do
    echo "== $L round $r"
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 120 python -u tools/occupancy.py $ARGS 2>&1 | grep "R=" || exit 1
  done
done
