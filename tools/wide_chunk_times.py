#!/usr/bin/env python3
"""Per-tile chunk timeline of the wide E-step (diagnostics): builds the engine with shader-clock stamps
(-DHMMBW_PHASE_TIMES -DHMMBW_CHUNK_TIMES) into hmm_training_amd/libhmmbw_wstamp.so unless present, runs
a cfg5-shaped workload and prints, over the waves of the last launch, the cycles per forward / backward
step of the steady chunks and the phase boundaries (shader clock; cycles, not seconds).

    python tools/wide_chunk_times.py [--R 4096,6250] [--T 400] [--N 64] [--K 1024]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", default="4096,6250")
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--ablate", default="0", help="comma-separated HMMBW_WIDE_ABLATE bit sets (4: no gamma rows, "
                                                  "8: no alpha_hat stores/loads, 16: no per-step barrier; wrong results)")
    ap.add_argument("--lib", default=None, help="a prebuilt stamped library (e.g. a compile-time ablation)")
    a = ap.parse_args()
    lib = a.lib or os.path.join(ROOT, "hmm_training_amd", "libhmmbw_wstamp.so")
    if not os.path.exists(lib) and not a.lib:
        from hmm_training_amd import build as B
        B.build(force=True, defines=["-DHMMBW_PHASE_TIMES", "-DHMMBW_CHUNK_TIMES", "-DHMMBW_WIDE_ABLATE"], out=lib,
                tag="wstamp")
    os.environ["HMMBW_LIB"] = lib
    import torch
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    T, N, K = a.T, a.N, a.K
    for R, abl in [(int(x), int(b)) for x in a.R.split(",") for b in a.ablate.split(",")]:
        rng = np.random.default_rng(5)
        sym = rng.integers(0, K, size=R * T).astype(np.int32)
        pi, A, B = default_initial_params(N, K)
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
        B = rng.dirichlet(np.full(K, 2.0), size=N)
        with BaumWelchEngine(N, K, topology="dense") as e:
            e.set_observations(offsets=np.arange(R + 1, dtype=np.int64) * T, symbols=sym)
            e.set_params(pi, A, B)
            e._lib.hmmbw_set_option(e._ctx, 2, abl)  # HMMBW_OPT_ABLATE (diagnostics)
            e.reset(0.0, 1 << 40)
            e.enqueue_iterations(3)
            torch.cuda.synchronize()
            tiles = (R + 15) // 16
            nw = tiles * ((N + 15) // 16)
            buf = (ctypes.c_ulonglong * (128 * nw))()
            fn = e._lib.hmmbw_debug_wide_chunk_times
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
            assert fn(buf, nw) == 0
        st = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 2, 64).astype(np.int64)
        nch = (T + 7) // 8
        t0 = st[:, 0, 62].min()
        fwd = np.diff(st[:, 0, 1:nch], axis=1) / 8.0          # steady forward chunks, cycles per step
        bwd = -np.diff(st[:, 1, 1:nch - 1], axis=1) / 8.0     # backward chunks run c = nch-1 .. 0
        q = lambda x: f"p10 {np.percentile(x, 10):7.0f}  p50 {np.percentile(x, 50):7.0f}  p90 {np.percentile(x, 90):7.0f}"
        print(f"==== R={R} ablate={abl}: {tiles} tiles, {nw} waves")
        print(f"forward  cycles/step  {q(fwd)}")
        print(f"backward cycles/step  {q(bwd)}")
        for name, v in (("start", st[:, 0, 62]), ("forward end", st[:, 0, 61]), ("backward end", st[:, 1, 62]),
                        ("kernel end", st[:, 1, 63])):
            print(f"{name:13s} rel cycles  {q(v - t0)}")
        dur = st[:, 1, 63] - st[:, 0, 62]
        print(f"tile duration cycles  {q(dur)}  (max {dur.max()})")


if __name__ == "__main__":
    main()
