#!/bin/bash
# after the r4h parity run: dense cfg3 / cfg5 / LR bench lines of the new kernels (compared with profiles/r3),
# LR per-step costs, the synced protocol (live mirror) and the peer all-reduce's 1-GPU cost
set -uo pipefail
OUT=gpurun_out/r4h
mkdir -p $OUT
show() { grep '"metric"' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', 'value %.4g' % d['value'], 'ms/step %.2f us' % (d['ms_per_step']*1000), 'kernel %.2f us' % (r.get('kernel_ms', 0)*1000), 'synced', d.get('synced'))"; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --topology dense --steps 100 --warmup 5 --no-cpu-baseline --no-synced > $OUT/bench_dense_$r.log 2>&1 || { tail -20 $OUT/bench_dense_$r.log; exit 1; }
  show $OUT/bench_dense_$r.log dense
  timeout -k 10 200 python -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-synced > $OUT/bench_cfg5_$r.log 2>&1 || { tail -20 $OUT/bench_cfg5_$r.log; exit 1; }
  show $OUT/bench_cfg5_$r.log cfg5
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
show $OUT/bench.log lr
timeout -k 10 300 python -u tools/multirank_overhead.py --modes single,native,split,peer > $OUT/overhead_cfg3.jsonl 2> $OUT/overhead_cfg3.err || { tail $OUT/overhead_cfg3.err; exit 1; }
grep '^{' $OUT/overhead_cfg3.jsonl
# per-step costs of the LR kernel: forward-only (ablate 2) and full launches at T = 200 and 800, one and two
# waves per SIMD (the T slope is the per-step cost, the intercept the prologue + flush)
for T in 200 800; do
  echo "== LR T=$T"
  timeout -k 10 180 python -u tools/occupancy.py --Rs 8192,16384 --T $T --ablate 0,2 --iters 20 2>&1 | grep "R=" || exit 1
done
