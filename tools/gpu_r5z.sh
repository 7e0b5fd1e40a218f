#!/bin/bash
# Round 5: the wide kernels built with the memory-clause scheduler: every wide parity test, then cfg5 shard and whole.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py \
  -k "cfg5 or wide or work_queue or 64 or 48 or 33 or 24 or 17 or 40 or 49" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for W in "--workload cfg5 --steps 50 --warmup 5" "--workload cfg5 --R 50000 --steps 5 --warmup 1"; do
  timeout -k 10 300 python -u bench.py $W --no-cpu-baseline --no-synced > $O/b.log 2>&1 || exit 1
  python3 - $O/b.log "$W" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:50s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.1f}us estep={r['model']['kernel_ms']*1e3:.1f}us")
PY
done
