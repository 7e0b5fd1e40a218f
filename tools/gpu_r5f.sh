#!/bin/bash
# Round 5: cfg4-shard spread map (xact 3) A/B, dense every-z_t store A/B, then the cfg3 profiles (part a).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5f
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us kernel={d['roofline']['kernel_ms']*1e3:.2f}us map={d['roofline'].get('launch_map')}")
PY
}
for X in default 3; do
  step cfg4 xact=$X
  if [ $X = default ]; then E=""; else E="HMMBW_XACT=$X"; fi
  env $E timeout -k 10 200 python -u bench.py --workload cfg4 --steps 200 --warmup 10 --no-cpu-baseline --no-synced > $O/cfg4_x$X.log 2>&1 || exit 1
  summ $O/cfg4_x$X.log "cfg4 xact=$X"
done
for L in libhmmbw.so libhmmbw_zf0.so; do
  step dense $L
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --topology dense --steps 200 --warmup 10 --no-cpu-baseline --no-synced > $O/dense_$L.log 2>&1 || exit 1
  summ $O/dense_$L.log "dense $L"
done
step profiles
timeout -k 10 900 bash tools/profile_all.sh r5 a > $O/profile_a.log 2>&1 || { tail -5 $O/profile_a.log; exit 1; }
step done
