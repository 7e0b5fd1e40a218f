"""Dense cfg3 (N=8, K=256, T=200, R=10,000): E-step time of the fp64-MFMA kernel vs the VALU kernel,
with ablations (bit 1: skip flush, bit 2: skip backward).  Diagnostics only."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params
R, T, N, K = 10000, 200, 8, 256
rng = np.random.default_rng(3)
sym = rng.integers(0, K, size=R * T).astype(np.int32)
off = np.arange(R + 1, dtype=np.int64) * T
pi, A, B = default_initial_params(N, K)
A = 0.5 * A + 0.5 * np.random.default_rng(3).dirichlet(np.ones(N), size=N)
for mfma in (2, 0):
    e = BaumWelchEngine(N, K, topology="dense")
    e._lib.hmmbw_set_option(e._ctx, 5, mfma)
    e.set_observations(offsets=off, symbols=sym)
    for ablate in (0, 1, 2, 3):
        e._lib.hmmbw_set_option(e._ctx, 2, ablate)
        e.set_params(pi, A, B); e.reset(0.0, 100); e.enqueue_iterations(2); torch.cuda.synchronize()
        e.timing(1); e.enqueue_iterations(10); ms, n = e.timing(0)
        sc = []
        for _ in range(5):
            torch.cuda.synchronize(); t0 = time.perf_counter(); e.score(); sc.append(time.perf_counter() - t0)
        print(f"mfma={mfma} ablate={ablate}: estep {ms / n * 1e3:8.1f} us  score incl. D2H {min(sc) * 1e6:8.1f} us", flush=True)
    e.close()
