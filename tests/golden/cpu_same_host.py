#!/usr/bin/env python3
"""Same-host CPU ratio: the reference NumPy path vs the oracle C restatement, timed on ONE host.

bench.py's cpu_baseline times the oracle on the GPU box's host cores, where the reference cannot run
(it does not travel).  Its ratio to the reference therefore used to divide by a rate measured on a
different CPU.  This script runs in the build container (where /root/reference is mounted read-only)
and times, on the same cfg3-shaped sample (T = 200, N = 8, K = 256, the left-to-right init, uniform
symbols, ONE EM iteration, hmm_training.py:265-541):

* the reference's own ``hmm_training`` (imported with the stand-ins of make_golden.py; N = 8 is driven
  through its warm-start path, hmm_training.py:275-287), one process = one core;
* the oracle (oracle/bw_oracle.c, log domain like the reference) on 1 thread and on every core of
  this host (OpenMP over utterances).

It writes profiles/<round>/cpu_same_host.json, which bench.py reads to report the same-host ratio
beside the cross-host one.  Test infrastructure: nothing of the reference travels, only the JSON.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/cpu_same_host.py [--round r4]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r4")
    ap.add_argument("--ref-R", type=int, default=20, help="sequences per reference run (survey: 20)")
    ap.add_argument("--ref-runs", type=int, default=3)
    args = ap.parse_args()

    import make_golden as MG  # imports the reference (build container only)
    from oracle import oracle as O

    T, N, K = 200, 8, 256
    pi, A, B = MG.left_to_right(N, K)
    rng = np.random.default_rng(3)

    # ---- reference: one process, one core (numpy single-threaded as in the survey), no trace hook ----
    import contextlib
    import io
    import tempfile
    ref_times = []
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "cwd"))
        model = MG.HC.HMMTrained(N, K, A, B, pi, "w")
        MG.HC.DataStorageHMM.save_hmm(model, base_dir=os.path.join(tmp, "Data", "Eighty-five-percent_20"),
                                      print_messages=False)
        os.chdir(os.path.join(tmp, "cwd"))
        try:
            for run in range(args.ref_runs):
                obs = [rng.integers(0, K, size=T).astype(np.int64) for _ in range(args.ref_R)]
                with contextlib.redirect_stdout(io.StringIO()):
                    t0 = time.perf_counter()
                    MG.HT.hmm_training(obs, N=N, M=K, epsilon=0.0, max_iterations=1, show_progress=True,
                                       word_name="w", load_initial_params=True)
                    ref_times.append(time.perf_counter() - t0)
        finally:
            os.chdir(cwd)
    ref_rate = args.ref_R / float(np.median(ref_times))

    # ---- oracle: 1 thread and all threads, same shape ----
    nth_all = len(os.sched_getaffinity(0))

    def oracle_rate(threads, R, reps=3):
        O.set_threads(threads)
        best = []
        for _ in range(reps):
            sym = rng.integers(0, K, size=R * T).astype(np.int64)
            off = np.arange(R + 1, dtype=np.int64) * T
            t0 = time.perf_counter()
            O.hmm_training(off, sym, N, K, 0.0, 1, pi, A, B)
            best.append(time.perf_counter() - t0)
        O.set_threads(1)
        return R / float(np.median(best))

    o1 = oracle_rate(1, 2_000)
    on = oracle_rate(nth_all, 20_000)
    out = {
        "host": cpu_model(), "cores_visible": nth_all, "python": platform.python_version(),
        "numpy": np.__version__,
        "sample": f"T={T}, N={N}, K={K}, left-to-right init (make_golden.left_to_right), uniform symbols, "
                  f"1 EM iteration; reference R={args.ref_R} x {args.ref_runs} runs (median), oracle R=2,000 on 1 "
                  f"thread and R=20,000 on {nth_all} threads (median of 3)",
        "reference_utt_per_s_1core": ref_rate,
        "oracle_utt_per_s_1thread": o1,
        f"oracle_utt_per_s_{nth_all}threads": on,
        "oracle_threads_all": nth_all,
        "ratio_oracle_vs_reference_per_core": o1 / ref_rate,
        "ratio_oracle_all_vs_reference_1core": on / ref_rate,
        "note": "both timed on this host back to back; bench.py divides the GPU box's oracle rate by this per-core "
                "ratio to estimate the reference's rate on the box's cores",
    }
    dst = os.path.join(ROOT, "profiles", args.round, "cpu_same_host.json")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=2)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main()
