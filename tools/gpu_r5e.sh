#!/bin/bash
# Round 5: paired-tile wide E-step — parity, then the cfg5-shard bench with and without pairs.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5e
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
step pytest
HMMBW_WIDE_PAIR=-1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py \
  -k "wide or cfg5_shard or cfg5_full_shape or work_queue or multirank" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for P in 1 0; do
  step bench cfg5 pair=$P
  HMMBW_WIDE_PAIR=$P timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline \
    --no-synced > $O/bench_cfg5_pair$P.log 2>&1 || exit 1
  python - $O/bench_cfg5_pair$P.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
rf = d["roofline"]
print(f"value={d['value']:.4g} ms/step={d['ms_per_step']:.4f} estep_ms={rf['model']['kernel_ms']:.4f} "
      f"estep+gather_ms={rf['kernel_ms']:.4f} frac={rf['frac']:.3f} map={rf['launch_map']}")
PY
done
step done
