"""E-step time of the left-to-right kernels (one vs two states per lane) against the sequence count
at T=200, N=8, K=256 (diagnostics).   python tools/sweep_lr2.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params
T, N, K = 200, 8, 256
pi, A, B = default_initial_params(N, K)
for R in [int(x) for x in os.environ.get("RS", "4096,8192,10000,16384").split(",")]:
    rng = np.random.default_rng(3)
    sym = rng.integers(0, K, size=R * T).astype(np.int32)
    off = np.arange(R + 1, dtype=np.int64) * T
    for pairs in (0, 1):
        e = BaumWelchEngine(N, K, topology="left_to_right")
        e._lib.hmmbw_set_option(e._ctx, 6, pairs)
        e.set_observations(offsets=off, symbols=sym); e.set_params(pi, A, B)
        e.reset(0.0, 1000); e.enqueue_iterations(3); torch.cuda.synchronize()
        e.timing(5)
        t0 = time.perf_counter(); e.enqueue_iterations(50); torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 50
        ms, n = e.timing(0)
        print(f"R={R:6d} pairs={pairs}: iteration {dt * 1e6:7.1f} us  estep {ms / n * 1e3:7.1f} us  -> {R / dt:.3e} utt/s/iter", flush=True)
        e.close()
