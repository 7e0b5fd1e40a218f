#!/bin/bash
# Build a variant library for on-box A/B timing: the release objects are reused except the listed
# units, recompiled with extra defines.   bash tools/variant_build.sh <name> "<units>" [defines...]
set -euo pipefail
NAME=$1; UNITS=$2; shift 2
mkdir -p hmm_training_amd/_obj/$NAME
cp -n hmm_training_amd/_obj/release/*.o hmm_training_amd/_obj/$NAME/ 2>/dev/null || true
DEFS=$(printf '"%s",' "$@")
python - <<PY
from hmm_training_amd import build as B
print(B.build(only="$UNITS".split(","), defines=[${DEFS%,}], out="hmm_training_amd/libhmmbw_$NAME.so", tag="$NAME"))
PY
