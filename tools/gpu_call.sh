#!/bin/bash
# One gpurun call from a step file (replaces the per-call gpu_r5*.sh scripts of round 5):
#   bash tools/gpu_call.sh <tag> <stepfile>
# Each non-comment line of the step file is:  <timeout_s> <name> <command ...>
# The command runs from the repo root under `timeout -k 10 <timeout_s>`, output to gpurun_out/<tag>/<name>.log.
# Exit status 0 continues; 1 (pytest assertion failures, or a probe's "not as expected") is reported and
# continues; anything else (a fault, abort, segfault, time limit) stops the call: nothing more touches the GPU.
set -uo pipefail
TAG=$1
STEPS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
worst=0
while read -r T NAME CMD; do
  [ -z "${T:-}" ] && continue
  case "$T" in \#*) continue ;; esac
  echo "[$(date +%T)] $NAME: $CMD"
  timeout -k 10 "$T" bash -c "$CMD" > "$OUT/$NAME.log" 2>&1
  rc=$?
  grep -E "passed|failed|error|Error|\{\"metric\"" "$OUT/$NAME.log" | tail -4
  echo "[$(date +%T)] $NAME rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $NAME (rc=$rc)"; exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done < "$STEPS"
exit $worst
