#!/bin/bash
# Round 5: the host-side fixed cost of the timed region (tools/sync_latency.py) under the default wait,
# HSA_ENABLE_INTERRUPT=0 and hipDeviceScheduleSpin; then bench.py at 20 and 200 steps.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5i
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
step sync default
timeout -k 10 120 python -u tools/sync_latency.py > $O/sync.log 2>&1 || exit 1
step sync nointerrupt
HSA_ENABLE_INTERRUPT=0 timeout -k 10 120 python -u tools/sync_latency.py >> $O/sync.log 2>&1 || exit 1
step sync spin
timeout -k 10 120 python -u tools/sync_latency.py --spin >> $O/sync.log 2>&1 || exit 1
grep -v amdgpu.ids $O/sync.log
for S in 20 200 20; do
  step bench steps=$S
  timeout -k 10 200 python -u bench.py --steps $S --warmup 10 --no-cpu-baseline --no-synced > $O/bench_s$S.log 2>&1 || exit 1
  python3 - $O/bench_s$S.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"steps={d['steps']} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us gpu/step={d['roofline']['gpu_ms_per_step']*1e3:.2f}us kernel={d['roofline']['kernel_ms']*1e3:.2f}us")
PY
done
step done
