"""Per-call costs of the drop-in training path (diagnostics): engine setup for one word (cfg1/cfg2
shape, 20 utterances), and the pipelined train() loop at cfg3 against the same iterations enqueued
back to back.     python tools/dropin_time.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.init()
torch.zeros(1, device="cuda")
from hmm_training_amd.engine import BaumWelchEngine  # noqa: E402
from hmm_training_amd.hmm_training import default_initial_params  # noqa: E402

rng = np.random.default_rng(0)
obs = [rng.integers(0, 256, size=int(t)) for t in rng.integers(40, 121, size=20)]
pi, A, B = default_initial_params(8, 256)
for rep in range(3):
    t = [time.perf_counter()]
    e = BaumWelchEngine(8, 256); t.append(time.perf_counter())
    e.set_observations(obs); t.append(time.perf_counter())
    e.set_params(pi, A, B); t.append(time.perf_counter())
    st = e.train(1e-6, 30); t.append(time.perf_counter())
    p = e.params(); t.append(time.perf_counter())
    e.close(); t.append(time.perf_counter())
    print("word (20 utt): create %.0f obs %.0f params %.0f train(%d it) %.0f get %.0f close %.0f us" %
          (*(1e6 * (b - a) for a, b in list(zip(t, t[1:]))[:3]), st.iterations, 1e6 * (t[4] - t[3]),
           1e6 * (t[5] - t[4]), 1e6 * (t[6] - t[5])), flush=True)

R, T = 10000, 200
sym = rng.integers(0, 256, size=R * T).astype(np.int32)
with BaumWelchEngine(8, 256) as e:
    e.set_observations(offsets=np.arange(R + 1, dtype=np.int64) * T, symbols=sym)
    for it in (20, 100):
        for rep in range(3):
            e.set_params(pi, A, B)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.reset(0.0, it)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            e.enqueue_iterations(it)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            e.status(0, 0)
            t3 = time.perf_counter()
            e.set_params(pi, A, B)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            st = e.train(0.0, it)
            t5 = time.perf_counter()
            print("cfg3 %3d it: reset+sync %.0f us, enqueue+sync %.1f us/it, final status %.0f us | train() %.1f us/it" %
                  (it, 1e6 * (t1 - t0), 1e6 * (t2 - t1) / it, 1e6 * (t3 - t2), 1e6 * (t5 - t4) / it), flush=True)
