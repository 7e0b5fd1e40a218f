import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hmm_training_amd.engine import BaumWelchEngine, to_csr
from oracle import oracle as O
for N, K in ((8, 16), (9, 16), (16, 16)):
    rng = np.random.default_rng(1000 * N + K)
    lengths = rng.integers(1, 91, size=37); lengths[0] = 90
    obs = [rng.integers(0, K, size=int(t)) for t in lengths]
    A = rng.dirichlet(np.ones(N), size=N); pi = rng.dirichlet(np.ones(N)); B = rng.dirichlet(np.full(K, 0.5), size=N)
    off, sym = to_csr(obs)
    ref = O.forward_loglik(off, sym.astype(np.int64), N, K, pi, A, B)
    with BaumWelchEngine(N, K, topology="dense") as e:
        e.set_observations(obs); e.set_params(pi, A, B)
        sc = e.score()
        e.reset(0.0, 1); e.enqueue_iterations(1); st, recs = e.status(0, 1)
        ll = e.loglik()
    bad = np.where(~np.isclose(sc, ref, rtol=1e-9))[0]
    bad2 = np.where(~np.isclose(ll, ref, rtol=1e-9))[0]
    order = np.argsort(-lengths, kind="stable")
    print(f"N={N}: score bad {bad.tolist()} estep bad {bad2.tolist()}; L {recs[0][0]:.9f} vs {O.lse(ref):.9f}")
    print("   lengths of bad:", lengths[bad2].tolist(), " slot positions:", [int(np.where(order == b)[0][0]) for b in bad2])
