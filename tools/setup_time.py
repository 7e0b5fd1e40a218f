import time, numpy as np, sys, os
sys.path.insert(0, os.getcwd())
import torch
torch.cuda.init(); torch.zeros(1, device="cuda")
from hmm_training_amd.engine import BaumWelchEngine
from hmm_training_amd.hmm_training import default_initial_params
rng = np.random.default_rng(0)
obs = [rng.integers(0, 256, size=int(t)) for t in rng.integers(40, 121, size=20)]
pi, A, B = default_initial_params(8, 256)
for rep in range(3):
    t = [time.perf_counter()]
    e = BaumWelchEngine(8, 256); t.append(time.perf_counter())
    e.set_observations(obs); t.append(time.perf_counter())
    e.set_params(pi, A, B); t.append(time.perf_counter())
    st = e.train(1e-6, 2); t.append(time.perf_counter())
    p = e.params(); t.append(time.perf_counter())
    e.close(); t.append(time.perf_counter())
    print("create %.0f obs %.0f params %.0f train %.0f get %.0f close %.0f us" % tuple(1e6*(b-a) for a, b in zip(t, t[1:])), flush=True)
