"""On-box A/B of library variants through bench.py (pre-warmed, HIP-event GPU time per EM iteration),
interleaved in rounds so that every variant sees the same box and clocks.

    python tools/ab_bench.py --libs libhmmbw.so,libhmmbw_x.so,libhmmbw.so:HMMBW_XACT=1 --cases lr,dense,cfg4,t8 [--rounds 2]
(';' separates library specs when one carries several settings: --libs 'libhmmbw.so;libhmmbw.so:A=1,B=2')

cases: lr (cfg3 left-to-right), lrH (cfg3 skewed symbols), dense (cfg3 dense), cfg4 (the 12,500 shard),
t8 (T = 8 at 8,192 sequences: the fixed cost per launch), cfg5 (the wide shard, 6,250 x 400), r8k / r4k (8,192 /
4,096 sequences at T = 200: one sequence group per SIMD / on every other SIMD, no extra groups).
Prints one line per (round, case, lib) and a median summary per (case, lib)."""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {
    "lr": [],
    "lrH": ["--symbols", "H"],
    "dense": ["--topology", "dense"],
    "cfg4": ["--workload", "cfg4"],
    "t8": ["--R", "8192", "--T", "8"],
    "cfg5": ["--workload", "cfg5"],
    "r8k": ["--R", "8192"],
    "r4k": ["--R", "4096"],
}


def run(spec, case, steps):
    """spec: a library file name, optionally with environment settings: libhmmbw.so:HMMBW_XACT=1,HMMBW_JOIN=0"""
    lib, _, envs = spec.partition(":")
    env = dict(os.environ, HMMBW_LIB=os.path.join(ROOT, "hmm_training_amd", lib))
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    st = steps if case != "cfg5" else max(10, steps // 20)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-synced",
           "--steps", str(st), "--warmup", "5", *CASES[case]]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        sys.stderr.write(out.stdout[-3000:] + out.stderr[-3000:])
        raise SystemExit(out.returncode)
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    rf = d.get("roofline", {})
    gpu_us = 1e3 * rf.get("kernel_ms", float("nan"))
    return gpu_us, 1e3 * d["ms_per_step"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--cases", default="lr")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    libs = a.libs.split(";") if ";" in a.libs else a.libs.split(",")
    res = {}
    for r in range(a.rounds):
        for case in a.cases.split(","):
            for lib in libs:
                g, w = run(lib, case, a.steps)
                res.setdefault((case, lib), []).append(g)
                print(f"round {r} {case:6s} {lib:28s} gpu/iter {g:9.2f} us  wall/iter {w:9.2f} us", flush=True)
    print("# median GPU us per iteration")
    for (case, lib), v in res.items():
        print(f"{case:6s} {lib:28s} {statistics.median(v):9.2f}  ({', '.join(f'{x:.2f}' for x in v)})")


if __name__ == "__main__":
    main()
