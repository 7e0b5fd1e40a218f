#!/bin/bash
# Round-4 measurements: multi-rank overheads on one GPU (RCCL 1-rank vs peer all-reduce), the counter list.
set -uo pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || echo "counter list failed"
timeout -k 10 300 python -u tools/multirank_overhead.py --steps 300 > $OUT/overhead_cfg3.jsonl 2>$OUT/overhead_cfg3.err || exit 1
cat $OUT/overhead_cfg3.jsonl
timeout -k 10 300 python -u tools/multirank_overhead.py --steps 300 --R 12500 --modes single,native,split,peer > $OUT/overhead_cfg4.jsonl 2>$OUT/overhead_cfg4.err || exit 1
cat $OUT/overhead_cfg4.jsonl
timeout -k 10 300 python -u tools/multirank_overhead.py --steps 30 --workload cfg5 --modes single,native,split,peer > $OUT/overhead_cfg5.jsonl 2>$OUT/overhead_cfg5.err || exit 1
cat $OUT/overhead_cfg5.jsonl
timeout -k 10 300 python -u bench.py --gpus 2 --R 10000 --steps 50 --warmup 5 --dist-backend gloo --allreduce peer --no-synced > $OUT/bench_2rank_peer.log 2>&1 || exit 1
tail -1 $OUT/bench_2rank_peer.log | cut -c1-600
