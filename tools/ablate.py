"""Time E-step variants at the bench workload with fresh parameters before every timed launch
(diagnostics; ablated results are wrong by construction)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params
R, T, N, K = (int(os.environ.get(k, d)) for k, d in (("R", 10000), ("T", 200), ("N", 8), ("K", 256)))
rng = np.random.default_rng(3)
sym = rng.integers(0, K, size=R * T).astype(np.int32)
off = np.arange(R + 1, dtype=np.int64) * T
for topo in os.environ.get("TOPOS", "left_to_right,dense").split(","):
    pi, A, B = default_initial_params(N, K)
    B = np.random.default_rng(5).dirichlet(np.full(K, 2.0), size=N)
    if topo == "dense":
        A = 0.5 * A + 0.5 * np.random.default_rng(3).dirichlet(np.ones(N), size=N)
    e = BaumWelchEngine(N, K, topology=topo)
    e.set_observations(offsets=off, symbols=sym)
    for ablate in [int(x) for x in os.environ.get("ABL", "0,1,2,3").split(",")]:
        e._lib.hmmbw_set_option(e._ctx, 2, ablate)
        e.set_params(pi, A, B); e.reset(0.0, 100); e.enqueue_iterations(1); torch.cuda.synchronize()
        tot, n = 0.0, 0
        for rep in range(10):
            e.set_params(pi, A, B); e.reset(0.0, 100)
            e.timing(1); e.enqueue_iterations(1); ms, k = e.timing(0)
            tot += ms; n += k
        sc = []
        for rep in range(5):
            e.set_params(pi, A, B)
            torch.cuda.synchronize(); t0 = time.perf_counter(); e.score(); sc.append(time.perf_counter() - t0)
        print(f"R={R} {topo:14s} ablate={ablate}: estep {tot / n * 1e3:8.1f} us   (score incl. D2H min {min(sc) * 1e6:8.1f} us)", flush=True)
    e.close()
