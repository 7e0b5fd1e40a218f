#!/usr/bin/env python3
"""BASELINE cfg2 measurement: 10 word models x 20 utterances (T ~ U[40, 120]), N=8, K=256, one MI355X.

Compares, per EM iteration of ALL ten models:
  grouped     one k_estep_small_group launch per iteration for the ten models (hmmbw_group_iterate);
  sequential  the reference's word-by-word order (HMM/main.py:147-152): ten single-model runs;
  cpu oracle  oracle/bw_oracle.c (log domain, 1 thread) on the same ten words (baseline only);
plus the end-to-end train loop (EngineGroup.train vs BaumWelchEngine.train per word, 100 iterations,
epsilon 0 so no early stop), which includes the host's status polls.
Prints one JSON line.   python tools/bench_cfg2.py [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def words(n=10, R=20, N=8, K=256):
    from hmm_training_amd.hmm_training import default_initial_params
    out = []
    for w in range(n):
        rng = np.random.default_rng(2 + w)  # cfg2 seeds 2..11, one per word
        pi, A, B = default_initial_params(N, K)
        hot = rng.dirichlet(np.full(K, 0.3))
        obs = [rng.choice(K, size=int(t), p=hot) for t in rng.integers(40, 121, size=R)]
        out.append((obs, pi, A, B))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from hmm_training_amd.engine import BaumWelchEngine, EngineGroup
    N, K = 8, 256
    ws = words()
    n_utt = sum(len(w[0]) for w in ws)

    def engines():
        es = []
        for obs, pi, A, B in ws:
            e = BaumWelchEngine(N, K, device=0)
            e.set_observations(obs)
            e.set_params(pi, A, B)
            e.reset(0.0, 10 ** 9)
            es.append(e)
        return es

    res = {"workload": "cfg2: 10 words x 20 utterances, T~U[40,120], N=8, K=256, left_to_right", "utterances": n_utt}
    # grouped
    es = engines()
    g = EngineGroup(es)
    g.enqueue_iterations(5)
    torch.cuda.synchronize()
    g.timing(1)
    t0 = time.perf_counter()
    g.enqueue_iterations(args.iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, kn = g.timing(0)
    res["grouped"] = {"us_per_iter": 1e6 * dt / args.iters, "utt_per_s_iter": n_utt * args.iters / dt,
                      "kernel_us": 1e3 * kms / max(kn, 1), "launches_per_iter": 1}
    g.close()
    for e in es:
        e.close()
    # sequential, word by word
    es = engines()
    for e in es:
        e.enqueue_iterations(5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in es:
        e.enqueue_iterations(args.iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["sequential"] = {"us_per_iter": 1e6 * dt / args.iters, "utt_per_s_iter": n_utt * args.iters / dt,
                         "launches_per_iter": len(es)}
    for e in es:
        e.close()
    # end-to-end train loops (status polls included), 100 iterations each
    es = engines()
    g = EngineGroup(es)
    t0 = time.perf_counter()
    g.train(0.0, 100)
    res["train_grouped_ms"] = 1e3 * (time.perf_counter() - t0)
    g.close()
    for e in es:
        e.close()
    es = engines()
    t0 = time.perf_counter()
    for e in es:
        e.train(0.0, 100)
    res["train_sequential_ms"] = 1e3 * (time.perf_counter() - t0)
    for e in es:
        e.close()
    if not args.no_cpu:
        from oracle import oracle as O
        t0 = time.perf_counter()
        for obs, pi, A, B in ws:
            off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
            O.hmm_training(off, np.concatenate(obs).astype(np.int64), N, K, 0.0, 1, pi, A, B)
        dt = time.perf_counter() - t0
        res["cpu_oracle_1thread"] = {"us_per_iter": 1e6 * dt, "utt_per_s_iter": n_utt / dt}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
