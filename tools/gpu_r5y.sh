#!/bin/bash
# Round 5: LLVM scheduler strategies for the wide kernels (libhmmbw_wilp.so max-ilp, libhmmbw_wmcl.so
# max-memory-clause) against the default, cfg5 shard, alternating; parity of the faster first.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5y
mkdir -p $O
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.1f}us estep={r['model']['kernel_ms']*1e3:.1f}us")
PY
}
for rep in 1 2; do
  for L in libhmmbw.so libhmmbw_wilp.so libhmmbw_wmcl.so; do
    HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --workload cfg5 --steps 50 --warmup 5 --no-cpu-baseline --no-synced > $O/x.log 2>&1 || exit 1
    summ $O/x.log "$L"
  done
done
