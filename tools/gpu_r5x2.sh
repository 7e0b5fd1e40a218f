#!/bin/bash
# Round 5: LLVM iterative scheduler strategies for the N = 8 small kernels (libhmmbw_slat.so iterative-lat,
# libhmmbw_smin.so iterative-minreg) against the default, LR and dense cfg3, alternating.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5x2
mkdir -p $O
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:28s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
for rep in 1 2; do
  for L in libhmmbw.so libhmmbw_slat.so libhmmbw_smin.so; do
    for TOPO in left_to_right dense; do
      HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 300 --topology $TOPO --no-cpu-baseline --no-synced > $O/x.log 2>&1 || exit 1
      summ $O/x.log "$L $TOPO"
    done
  done
done
