#!/bin/bash
# A/B of the LR cfg3 E-step: the default library and variants named on the command line
#   bash tools/gpu_ab.sh <tag> [libhmmbw_<variant>.so ...]
set -uo pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for lib in libhmmbw.so "$@"; do
  for topo in left_to_right dense; do
    HMMBW_LIB=$PWD/hmm_training_amd/$lib timeout -k 10 120 python -u bench.py --topology $topo --no-cpu-baseline --no-synced --steps 50 --warmup 5 > "$OUT/${lib%.so}_$topo.log" 2>&1 || { echo "bench $lib $topo failed"; tail -20 "$OUT/${lib%.so}_$topo.log"; exit 1; }
    python - "$OUT/${lib%.so}_$topo.log" "$lib" "$topo" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:28s} {sys.argv[3]:14s} value={d['value']:.4g} ms/step={d['ms_per_step']*1000:.1f}us kernel={d['roofline']['kernel_ms']*1000:.1f}us")
PY
  done
done
