"""Wide-kernel (k_estep_mfma) cost breakdown at the cfg5 shard (6,250 x 400, N=64, K=1024, dense):
E-step kernel time per ablation of the diagnostics build (HMMBW_LIB=hmm_training_amd/libhmmbw_wabl.so,
-DHMMBW_WIDE_ABLATE; ablated results are wrong by construction).
    ablate bits: 2 backward skipped, 4 no gamma-row stores, 8 no alpha_hat checkpoint stores/loads,
                 16 no per-step barrier
    HMMBW_LIB=hmm_training_amd/libhmmbw_wabl.so python tools/ablate_wide.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params

R, T, N, K = (int(os.environ.get(k, d)) for k, d in (("R", 6250), ("T", 400), ("N", 64), ("K", 1024)))
rng = np.random.default_rng(5)
sym = rng.integers(0, K, size=R * T).astype(np.int32)
off = np.arange(R + 1, dtype=np.int64) * T
pi, A, B = default_initial_params(N, K)
A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
B = rng.dirichlet(np.full(K, 2.0), size=N)
e = BaumWelchEngine(N, K, topology="dense")
e.set_observations(offsets=off, symbols=sym)
for ablate in [int(x) for x in os.environ.get("ABL", "0,2,4,8,12,16,28,10,18").split(",")]:
    e._lib.hmmbw_set_option(e._ctx, 2, ablate)
    e.set_params(pi, A, B); e.reset(0.0, 100); e.enqueue_iterations(1); torch.cuda.synchronize()
    tot, n = 0.0, 0
    for rep in range(5):
        e.set_params(pi, A, B); e.reset(0.0, 100)
        e.timing(1); e.enqueue_iterations(1); ms, k = e.timing(0)
        tot += ms; n += k
    print(f"cfg5 ablate={ablate:2d}: E-step launch {tot / n * 1e3:8.1f} us", flush=True)
e.close()
