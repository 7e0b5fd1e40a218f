#!/bin/bash
# Round 5 diagnostics: every emission LDS read of the small kernels hits row 0 (libhmmbw_emr0.so,
# -DHMMBW_DIAG_EMROW0: broadcast, no bank conflicts; results wrong) - what conflict-free emission reads could gain.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:28s} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
mkdir -p gpurun_out/r5ae
for rep in 1 2; do
  for L in libhmmbw.so libhmmbw_emr0.so; do
    for TOPO in left_to_right dense; do
      HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 200 --topology $TOPO --no-cpu-baseline --no-synced --no-kernel-timing > gpurun_out/r5ae/x.log 2>&1 || exit 1
      summ gpurun_out/r5ae/x.log "$L $TOPO"
    done
  done
done
