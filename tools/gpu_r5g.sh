#!/bin/bash
# Round 5: dense 4-chain dot A/B; xi offload (estep_mfma.hpp xi_offload_units) parity, then the cfg5-shard A/B (off / on, unit sizes).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5g
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[$(date +%T)] $*"; }
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:24s} value={d['value']:.4g} ms/step={d['ms_per_step']:.4f} kernel={d['roofline']['kernel_ms']*1e3:.2f}us map={d['roofline'].get('launch_map')}")
PY
}
step parity
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_wide_xi_offload_timeout_is_an_error \
  tests/test_gpu_fullsize.py::test_xi_offload_narrow_tiles_vs_oracle \
  tests/test_gpu_fullsize.py::test_cfg5_shard_xi_offload_full_size_vs_oracle \
  tests/test_gpu_fullsize.py::test_cfg5_shard_full_size_vs_oracle \
  tests/test_gpu_parity.py::test_wide_work_queue_timeout_is_an_error > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
for X in 0 -1:40 -1:24 -1:80 0; do
  M=${X%%:*}; S=${X#*:}; [ "$S" = "$X" ] && S=40
  step cfg5 xoff=$M steps=$S
  HMMBW_WIDE_XOFF=$M HMMBW_XOFF_STEPS=$S timeout -k 10 200 python -u bench.py --workload cfg5 --steps 100 --warmup 5 \
    --no-cpu-baseline --no-synced > $O/cfg5_x${M}_s$S.log 2>&1 || exit 1
  summ $O/cfg5_x${M}_s$S.log "cfg5 xoff=$M steps=$S"
done
for L in libhmmbw.so libhmmbw_dot4.so libhmmbw.so libhmmbw_dot4.so; do
  step dense $L
  HMMBW_LIB=$R/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --topology dense --steps 200 --warmup 10 --no-cpu-baseline --no-synced > $O/dense_$L.log 2>&1 || exit 1
  summ $O/dense_$L.log "dense $L"
done
step done
