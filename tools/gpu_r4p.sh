#!/bin/bash
# A/B: alpha_hat with nontemporal stores and loads (gamma rows nontemporal in both), cfg5 shard, interleaved
set -uo pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
for r in 1 2 3; do
  for L in libhmmbw.so libhmmbw_nt.so; do
    HMMBW_LIB=$PWD/hmm_training_amd/$L timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/cfg5_${L%.so}_$r.log 2>&1 || { tail -20 $OUT/cfg5_${L%.so}_$r.log; exit 1; }
    grep '"metric"' $OUT/cfg5_${L%.so}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$L', 'value %.4g ms/step %.1f us kernel %.1f us estep %.1f us' % (d['value'], d['ms_per_step']*1e3, r['kernel_ms']*1e3, r['bounds']['simd_mfma']['kernel_ms']*1e3))"
  done
done
