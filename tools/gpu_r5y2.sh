#!/bin/bash
# Round 5: wide kernels with the iterative-minreg scheduler (libhmmbw_wmin.so, 23 spills) against the release
# (max-memory-clause, 31 spills), cfg5 shard alternating; then parity of the variant.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5y2
mkdir -p $O
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.1f}us estep={r['model']['kernel_ms']*1e3:.1f}us")
PY
}
for rep in 1 2 3; do
  for L in libhmmbw.so libhmmbw_wmin.so; do
    HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --workload cfg5 --steps 50 --warmup 5 --no-cpu-baseline --no-synced > $O/x.log 2>&1 || exit 1
    summ $O/x.log "$L"
  done
done
