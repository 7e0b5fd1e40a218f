"""E-step time per iteration vs sequence count (occupancy curve) and with the diagnostics ablations
(bit 0: no statistics flush, bit 1: no backward sweep; results wrong by construction), measured with one
event pair around a batch of back-to-back iterations (no per-launch events).  Diagnostics only.

    python tools/occupancy.py [--Rs 1024,4096,...] [--topology left_to_right] [--ablate 0,1,2,3]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Rs", default="1024,2048,4096,8192,10000,12500,16384,20480,32768")
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--N", type=int, default=8)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--topology", default="left_to_right")
    ap.add_argument("--ablate", default="0")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--copies", type=int, default=0, help="statistics copies (0: the engine default)")
    a = ap.parse_args()
    import torch
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    T, N, K = a.T, a.N, a.K
    for R in [int(x) for x in a.Rs.split(",")]:
        rng = np.random.default_rng(3)
        sym = rng.integers(0, K, size=R * T).astype(np.int32)
        pi, A, B = default_initial_params(N, K)
        B = rng.dirichlet(np.full(K, 2.0), size=N)
        if a.topology == "dense":
            A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
        kw = {"stat_copies": a.copies} if a.copies else {}
        with BaumWelchEngine(N, K, topology=a.topology, **kw) as e:
            e.set_observations(offsets=np.arange(R + 1, dtype=np.int64) * T, symbols=sym)
            # steady state: back-to-back iterations with the merged M-step
            e.set_params(pi, A, B)
            e.reset(0.0, 1 << 40)
            e.enqueue_iterations(5)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            e.enqueue_iterations(a.iters)
            e1.record()
            torch.cuda.synchronize()
            row = [f"steady {1000.0 * e0.elapsed_time(e1) / a.iters:7.2f} us |"]
            # isolated launches from fresh parameters (tables built from B^T, no merged M-step), per ablation
            for abl in [int(x) for x in a.ablate.split(",")]:
                e._lib.hmmbw_set_option(e._ctx, 2, abl)
                ts = []
                for rep in range(10):
                    e.set_params(pi, A, B)
                    e.reset(0.0, 1 << 40)
                    torch.cuda.synchronize()
                    e0.record()
                    e.enqueue_iterations(1)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(1000.0 * e0.elapsed_time(e1))
                row.append(f"isolated ablate={abl}: {np.median(ts):7.2f} us")
            e._lib.hmmbw_set_option(e._ctx, 2, 0)
            waves = (R + 64 // 8 - 1) // (64 // 8)
            print(f"R={R:6d} waves={waves:6d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
