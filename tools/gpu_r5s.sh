#!/bin/bash
# Round 5: left-to-right split extra waves (libhmmbw_splr.so) at xact 1 / 2 and priorities 0 / 1 / 2 against
# the release's left-to-right defaults.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5s
mkdir -p $O
export PYTHONUNBUFFERED=1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:28s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={r.get('launch_map',{}).get('workgroups')}/{r.get('launch_map',{}).get('extra_waves')}")
PY
}
timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-synced > $O/rel.log 2>&1 || exit 1
summ $O/rel.log "release"
for X in 1 2; do
  for P in 0 1 2; do
    HMMBW_LIB=$R/hmm_training_amd/libhmmbw_splr.so HMMBW_XACT=$X HMMBW_PRIO=$P timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-synced > $O/s_x${X}_p$P.log 2>&1 || exit 1
    summ $O/s_x${X}_p$P.log "splr xact=$X prio=$P"
  done
done
timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-synced > $O/rel.log 2>&1 || exit 1
summ $O/rel.log "release"
