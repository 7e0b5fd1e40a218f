"""GPU debug: per-sequence forward log-likelihood of the engine vs the oracle for small shapes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hmm_training_amd.engine import BaumWelchEngine, to_csr
from oracle import oracle as O

def case(N, K, lengths, topo, safe=False, seed=0):
    rng = np.random.default_rng(seed)
    obs = [rng.integers(0, K, size=t) for t in lengths]
    if topo == "dense":
        A = rng.dirichlet(np.ones(N), size=N); pi = rng.dirichlet(np.ones(N))
    else:
        A = np.zeros((N, N))
        for i in range(N):
            A[i, i] = 0.6 if i + 1 < N else 1.0
            if i + 1 < N: A[i, i + 1] = 0.4
        pi = np.full(N, 0.1 / max(N - 1, 1)); pi[0] = 0.9
    B = rng.dirichlet(np.ones(K), size=N)
    off, sym = to_csr(obs)
    ref = O.forward_loglik(off, sym.astype(np.int64), N, K, pi, A, B)
    with BaumWelchEngine(N, K, topology=topo, safe_scaling=safe) as e:
        e.set_observations(obs); e.set_params(pi, A, B)
        sc = e.score()
        e.reset(0.0, 1); e.enqueue_iterations(1); st, recs = e.status(0, 1)
        ll = e.loglik()
    print(f"N={N} K={K} {topo} safe={safe} T={lengths}")
    print("   oracle", np.round(ref, 6))
    print("   score ", np.round(sc, 6))
    print("   estep ", np.round(ll, 6), " L", recs[0][0], "vs", O.lse(ref))

for N in (8, 9, 16):
    case(N, 16, [5], "dense")
    case(N, 16, [12, 7, 5, 3], "dense")
    case(N, 16, [12, 7, 5, 3], "dense", safe=True)
    case(N, 16, [12, 12, 12, 12], "left_to_right")
