#!/bin/bash
# two ranks on one GPU: bench.py over gloo (RCCL refuses two ranks on one card), peer all-reduce leg
set -uo pipefail
OUT=gpurun_out/bench2
mkdir -p $OUT
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 10 --dist-backend gloo > $OUT/bench2.json 2> $OUT/bench2.err || { tail -30 $OUT/bench2.err; exit 1; }
tail -1 $OUT/bench2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['comm'])"
