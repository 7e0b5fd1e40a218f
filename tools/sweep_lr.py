"""LR E-step at warm clocks over R (the occupancy curve) and over T at R = 10,000 and 8,192 (per-step slope and the
T-independent intercept), bench.py --R / --T, 200 steps each; one summary line per run (round 5: tools/gpu_r5ac.sh).
    python tools/sweep_lr.py [out.txt]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNS = ([(R, 200) for R in (1024, 4096, 8192, 9000, 10000, 11000, 12500, 16384)]
        + [(10000, T) for T in (8, 25, 50, 100, 200, 400)] + [(8192, T) for T in (8, 50, 200)])


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    for R, T in RUNS:
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--R", str(R), "--T", str(T), "--steps", "200",
               "--no-cpu-baseline", "--no-synced"]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
        if p.returncode != 0:
            sys.stderr.write(p.stdout[-2000:] + p.stderr[-2000:])
            raise SystemExit(p.returncode)
        d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
        r = d["roofline"]
        m = r.get("launch_map") or {}
        line = (f"R={R:<6d} T={T:<4d} value={d['value']:.4g} gpu/step={r['gpu_ms_per_step'] * 1e3:.2f}us "
                f"map={m.get('workgroups')}/{m.get('extra_waves')} joined={m.get('joined')} split={m.get('split_extra')}")
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()


if __name__ == "__main__":
    main()
