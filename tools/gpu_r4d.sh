#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
L=hmm_training_amd/libhmmbw_chunk.so
timeout -k 10 200 python -u tools/phase_times.py --lib $L --R 1024,8192,10000 > $OUT/chunk_lr.txt 2>&1 || exit 1
grep -E "R=|chunk cycles|clock|forward->|tables->|start->" $OUT/chunk_lr.txt
timeout -k 10 200 python -u tools/phase_times.py --lib $L --R 10000 --topology dense > $OUT/chunk_dense.txt 2>&1 || exit 1
grep -E "R=|chunk cycles|clock" $OUT/chunk_dense.txt
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --cpu-seconds 3 > $OUT/bench.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['synced'])"
