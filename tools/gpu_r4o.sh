#!/bin/bash
# the r4 profiles, part b (cfg5, cfg4 shard, cfg2, vq, bench lines)
set -uo pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
bash tools/profile_all.sh r4 b > $OUT/prof_b.log 2>&1 || { tail -20 $OUT/prof_b.log; exit 1; }
tail -5 $OUT/prof_b.log
