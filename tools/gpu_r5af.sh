#!/bin/bash
# Round 5 diagnostics: the small kernels without the B-numerator LDS histogram adds (libhmmbw_nohist.so,
# -DHMMBW_NO_HIST, results wrong): the histogram's share of the launch at warm clocks.
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
mkdir -p gpurun_out/r5af
for rep in 1 2; do
  for L in libhmmbw.so libhmmbw_nohist.so; do
    for TOPO in left_to_right dense; do
      HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 200 --topology $TOPO --no-cpu-baseline --no-synced --no-kernel-timing > gpurun_out/r5af/x.log 2>&1 || exit 1
      summ gpurun_out/r5af/x.log "$L $TOPO"
    done
  done
done
