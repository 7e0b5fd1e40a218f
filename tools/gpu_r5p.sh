#!/bin/bash
# Round 5: left-to-right with b-only LDS tables (libhmmbw_lrb.so, -DHMMBW_LR_PTAB=0) against the release.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5p
mkdir -p $O
export PYTHONUNBUFFERED=1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us gpu/step={r['gpu_ms_per_step']*1e3:.2f}us")
PY
}
HMMBW_LIB=$R/hmm_training_amd/libhmmbw_lrb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "cfg3_full_size or spread_extra or cfg4_shard or split_extra" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2 3; do
  for L in libhmmbw.so libhmmbw_lrb.so; do
    HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-synced > $O/lr_$L.log 2>&1 || exit 1
    summ $O/lr_$L.log "lr $L"
  done
done
for L in libhmmbw.so libhmmbw_lrb.so libhmmbw.so libhmmbw_lrb.so; do
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 120 python -u tools/steady_ablate.py --modes merged --R 8192 --T 8 2>&1 | grep merged
done
