#!/bin/bash
# wave-priority A/B of the wide kernel (cfg5) and the small one (cfg3); fixed-cost decomposition of the LR
# E-step (isolated launches at T = 8 / 40 / 200, ablations: 1 no statistics flush, 2 no backward, 3 neither)
set -uo pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_deterministic.py tests/test_gpu_fuzz.py tests/test_gpu_multirank.py tests/test_gpu_peer.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; fi
show() { grep '"metric"' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; b=r.get('bounds',{}).get('simd_mfma',{}); print('$2', 'value %.4g' % d['value'], 'ms/step %.2f us' % (d['ms_per_step']*1000), 'kernel %.2f us' % (r.get('kernel_ms', 0)*1000), 'estep %.2f us' % (b.get('kernel_ms', 0)*1000))"; }
# wide tiles per CU: R = 4,096 (256 tiles, one per CU) / 6,250 (391) / 8,192 (512, two per CU)
for R in 4096 6250 8192; do
  timeout -k 10 200 python -u bench.py --workload cfg5 --R $R --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/cfg5_R$R.log 2>&1 || { tail -20 $OUT/cfg5_R$R.log; exit 1; }
  show $OUT/cfg5_R$R.log "cfg5 R=$R"
done
for r in 1 2; do
  for P in 0 3 4 5; do
    HMMBW_PRIO=$P timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/cfg5_p${P}_$r.log 2>&1 || { tail -20 $OUT/cfg5_p${P}_$r.log; exit 1; }
    show $OUT/cfg5_p${P}_$r.log "cfg5 prio=$P"
  done
  for P in 0 1 2; do
    echo "== LR prio $P round $r"
    HMMBW_PRIO=$P timeout -k 10 120 python -u tools/occupancy.py --Rs 10000,12500 --ablate 0 --iters 100 2>&1 | grep "R=" || exit 1
  done
done
for T in 8 40 200; do
  echo "== LR T=$T"
  timeout -k 10 180 python -u tools/occupancy.py --Rs 1024,8192 --T $T --ablate 0,1,2,3 --iters 20 2>&1 | grep "R=" || exit 1
done
