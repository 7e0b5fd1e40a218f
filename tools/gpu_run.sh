#!/bin/bash
# One GPU call: a pytest selection, then (if pytest ended normally: all passed or assertion failures
# only, exit 0/1) bench.py lines.  Stops at the first abort / fault / time limit.
#   bash tools/gpu_run.sh <tag> "<pytest args>" ["<bench args>" ...]
set -uo pipefail
TAG=$1; shift
PYT=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rc=0
if [ -n "$PYT" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread $PYT > "$OUT/pytest.log" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
fi
i=0
for B in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py $B > "$OUT/bench_$i.log" 2>&1
  brc=$?
  tail -3 "$OUT/bench_$i.log"
  if [ $brc -ne 0 ]; then echo "bench exit $brc: stopping"; exit $brc; fi
done
exit $rc
