#!/bin/bash
# A/B of the wide (cfg5) E-step: the default library and variants, alternated twice
#   bash tools/gpu_ab_cfg5.sh <tag> [libhmmbw_<variant>.so ...]
set -uo pipefail
TAG=${1:-ab5}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in libhmmbw.so "$@"; do
    HMMBW_LIB=$PWD/hmm_training_amd/$lib timeout -k 10 150 python -u bench.py --workload cfg5 --no-cpu-baseline --no-synced --steps 10 --warmup 2 > "$OUT/${lib%.so}_$rep.log" 2>&1 || { echo "bench $lib failed"; tail -20 "$OUT/${lib%.so}_$rep.log"; exit 1; }
    python - "$OUT/${lib%.so}_$rep.log" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:28s} value={d['value']:.4g} ms/step={d['ms_per_step']*1000:.1f}us kernel={d['roofline']['kernel_ms']*1000:.1f}us")
PY
  done
done
