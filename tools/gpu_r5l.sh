#!/bin/bash
# Round 5: every bench line with the pre-warm (quick look: no CPU baseline, no synced legs).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5l
mkdir -p $O
export PYTHONUNBUFFERED=1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
print(f"{sys.argv[2]:12s} value={d['value']:.4g} ms/step={d['ms_per_step']*1e3:.2f}us gpu/step={r['gpu_ms_per_step']*1e3:.2f}us kernel={r['kernel_ms']*1e3:.2f}us model_kernel={r['model']['kernel_ms']*1e3:.2f}us")
PY
}
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline --no-synced > $O/$name.log 2>&1 || exit 1; summ $O/$name.log $name; }
run lr_cfg3
run dense_cfg3 --topology dense
run lrH_cfg3 --symbols H
run cfg4shard --workload cfg4
run cfg5 --workload cfg5 --steps 50 --warmup 5
timeout -k 10 200 python3 tools/phase_times.py --R 10000 > $O/phase_cfg3_warm.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/phase_times.py --R 8192 --T 8 > $O/phase_T8_warm.log 2>&1 || exit 1
grep -v amdgpu.ids $O/phase_cfg3_warm.log $O/phase_T8_warm.log
