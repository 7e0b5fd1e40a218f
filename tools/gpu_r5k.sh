#!/bin/bash
# Round 5: bench.py at 20 steps with the default pre-warm (200 ms) and without, host trace of the region.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5k
mkdir -p $O
export PYTHONUNBUFFERED=1
for P in 200 0 200 0; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 10 --prewarm-ms $P --trace-region --no-cpu-baseline --no-synced > $O/bench_p$P.log 2>&1 || exit 1
  grep "trace rank" $O/bench_p$P.log
  python3 - $O/bench_p$P.log $P <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"prewarm={sys.argv[2]:4s}ms steps={d['steps']} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us gpu/step={d['roofline']['gpu_ms_per_step']*1e3:.2f}us")
PY
done
timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --trace-region --no-cpu-baseline --no-synced > $O/bench_s200.log 2>&1 || exit 1
grep "trace rank" $O/bench_s200.log
