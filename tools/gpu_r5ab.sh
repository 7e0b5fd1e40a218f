#!/bin/bash
# Round 5: dense split knobs (libhmmbw_sp2.so): B's share of the chunks (HMMBW_SPLIT_NUM / 16) and priority mode 3
# (the extra waves prioritised until the split barrier), cfg3 dense, 300 steps, one box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5ab
mkdir -p $O
export HMMBW_LIB=$R/hmm_training_amd/libhmmbw_sp2.so
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:24s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
for P in 0; do
  for NUM in 4 6 7 8 9; do
    HMMBW_PRIO=$P HMMBW_SPLIT_NUM=$NUM timeout -k 10 200 python -u bench.py --steps 300 --topology dense --no-cpu-baseline --no-synced > $O/x.log 2>&1 || exit 1
    summ $O/x.log "prio=$P num=$NUM"
  done
done
HMMBW_PRIO=0 HMMBW_SPLIT_NUM=8 timeout -k 10 200 python -u bench.py --steps 300 --topology dense --no-cpu-baseline --no-synced > $O/x.log 2>&1 || exit 1
summ $O/x.log "prio=0 num=8 again"
