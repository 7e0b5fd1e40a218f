"""Per-iteration time vs number of statistics copies (bench workload)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params
R, T, N, K = int(os.environ.get("R", 10000)), 200, 8, 256
rng = np.random.default_rng(3)
sym = rng.integers(0, K, size=R * T).astype(np.int32)
off = np.arange(R + 1, dtype=np.int64) * T
pi, A, B = default_initial_params(N, K)
for topo in ("left_to_right", "dense"):
    if topo == "dense":
        A = 0.5 * A + 0.5 * np.random.default_rng(3).dirichlet(np.ones(N), size=N)
    for nc in [int(x) for x in os.environ.get("NCS", "1,4,8,16,32,64").split(",")]:
        e = BaumWelchEngine(N, K, topology=topo)
        e._lib.hmmbw_set_option(e._ctx, 3, nc)
        e.set_observations(offsets=off, symbols=sym); e.set_params(pi, A, B)
        e.reset(0.0, 1000); e.enqueue_iterations(3); torch.cuda.synchronize()
        e.timing(1)
        t0 = time.perf_counter(); e.enqueue_iterations(30); torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 30
        ms, n = e.timing(0)
        print(f"{topo:14s} copies={nc:3d}: iteration {dt * 1e6:7.1f} us  estep {ms / n * 1e3:7.1f} us", flush=True)
        e.close()
