#!/bin/bash
# Round 5: the joined map at the cfg4 shard (12,500 sequences: 539 extra groups, 4 per joined workgroup on 135 CUs)
# against separate workgroups (HMMBW_JOIN=0: 391 four-wave workgroups); parity first.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5ai
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py -k "cfg4_shard or cfg3_full_size_vs_oracle or spread_extra_waves_ragged" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
lm = r.get('launch_map', {})
print(f"{sys.argv[2]:24s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={lm.get('workgroups')}/{lm.get('extra_waves')} joined={lm.get('joined')}")
PY
}
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --workload cfg4 --steps 300 --no-cpu-baseline --no-synced > $O/$tag.log 2>&1 || exit 1; summ $O/$tag.log "$tag"; }
for i in 1 2; do
  run cfg4_join X=1
  run cfg4_sep HMMBW_JOIN=0
done
run cfg4_join_p0 HMMBW_PRIO=0
echo done
