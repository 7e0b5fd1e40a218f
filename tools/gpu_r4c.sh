#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_multirank.py tests/test_gpu_comm.py tests/test_bench.py > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/multirank_overhead.py --steps 300 --modes single,native,split,peer > $OUT/overhead_cfg3.jsonl 2>/dev/null || exit 1
cat $OUT/overhead_cfg3.jsonl
timeout -k 10 300 python -u tools/multirank_overhead.py --steps 30 --workload cfg5 --modes single,native,peer > $OUT/overhead_cfg5.jsonl 2>/dev/null || exit 1
cat $OUT/overhead_cfg5.jsonl
