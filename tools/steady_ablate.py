"""Steady-state EM iteration time (one event pair around a batch of back-to-back iterations) of the LR
E-step at a BASELINE shape, for the library in HMMBW_LIB and a list of diagnostics settings:
  merged      the production loop (M-step merged into the next E-step's prologue)
  noflush     ablate bit 0: no statistics flush (histogram + statistics atomics)
  unmerged0   merge off and no separate M-step kernel (ablate bit 2): tables built from B^T each launch
  unmerged0nf the same without the statistics flush
Results are wrong by construction except `merged`.  Diagnostics only.

    python tools/steady_ablate.py [--R 10000] [--T 200] [--iters 200] [--modes merged,noflush,...]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=10_000)
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--N", type=int, default=8)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--topology", default="left_to_right")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--modes", default="merged,noflush,unmerged0,unmerged0nf")
    a = ap.parse_args()
    import torch
    from hmm_training_amd._lib import OPT_ABLATE, OPT_MERGE_MSTEP
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    R, T, N, K = a.R, a.T, a.N, a.K
    rng = np.random.default_rng(3)
    sym = rng.integers(0, K, size=R * T).astype(np.int32)
    pi, A, B = default_initial_params(N, K)
    if a.topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    settings = {"merged": (1, 0), "noflush": (1, 1), "unmerged0": (0, 4), "unmerged0nf": (0, 5)}
    lib = os.path.basename(os.environ.get("HMMBW_LIB", "libhmmbw.so"))
    with BaumWelchEngine(N, K, topology=a.topology) as e:
        e.set_observations(offsets=np.arange(R + 1, dtype=np.int64) * T, symbols=sym)
        for mode in a.modes.split(","):
            merge, abl = settings[mode]
            e.set_option(OPT_MERGE_MSTEP, merge)
            e.set_option(OPT_ABLATE, abl)
            e.set_params(pi, A, B)
            e.reset(0.0, 1 << 40)
            e.enqueue_iterations(10)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            e.enqueue_iterations(a.iters)
            e1.record()
            torch.cuda.synchronize()
            print(f"{lib:28s} R={R} T={T} {a.topology:14s} {mode:12s} {1000.0 * e0.elapsed_time(e1) / a.iters:7.2f} us/iter",
                  flush=True)
        e.set_option(OPT_ABLATE, 0)


if __name__ == "__main__":
    main()
