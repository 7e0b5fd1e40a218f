#!/bin/bash
# Round 5: the joined map as the left-to-right default: the whole GPU suite, then the spread-map knobs on the
# joined map (HMMBW_PRIO x HMMBW_XACT, cfg3 left-to-right, 300 steps) and the release-map A/B (HMMBW_JOIN=0).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r5ah
mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu_tests.sh r5ah || exit 1
summ() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d['roofline']
lm = r.get('launch_map', {})
print(f"{sys.argv[2]:30s} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step']*1e3:.2f}us map={lm.get('workgroups')}/{lm.get('extra_waves')} joined={lm.get('joined')}")
PY
}
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 300 --no-cpu-baseline --no-synced > $O/$tag.log 2>&1 || exit 1; summ $O/$tag.log "$tag"; }
run join_p2_x2 HMMBW_PRIO=2 HMMBW_XACT=2
run join_p0_x2 HMMBW_PRIO=0 HMMBW_XACT=2
run join_p2_x1 HMMBW_PRIO=2 HMMBW_XACT=1
run join_p0_x1 HMMBW_PRIO=0 HMMBW_XACT=1
run join_p2_x3 HMMBW_PRIO=2 HMMBW_XACT=3
run release_map HMMBW_JOIN=0
run default X=1
run release_map2 HMMBW_JOIN=0
run default2 X=1
echo done
