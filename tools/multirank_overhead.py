#!/usr/bin/env python3
"""Per-iteration cost of the multi-rank EM path on ONE GPU: a 1-rank RCCL process group drives
hmmbw_estep -> all_reduce -> hmmbw_mstep (the path bench.py takes at N > 1) at the cfg3 workload,
next to the single-rank hmmbw_iterate path; also the host enqueue rate of that loop.
    python tools/multirank_overhead.py [--steps 200]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--R", type=int, default=10000)
    ap.add_argument("--modes", default="single,multirank,native,split,peer")
    ap.add_argument("--workload", default="cfg3", choices=["cfg3", "cfg5"])
    ap.add_argument("--copies", type=int, default=None, help="statistics copies (default: the library's)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    if a.workload == "cfg5" and a.R == 10000:
        a.R = 6250
    R, T, N, K = (a.R, 200, 8, 256) if a.workload == "cfg3" else (a.R, 400, 64, 1024)
    rng = np.random.default_rng(3)
    sym = rng.integers(0, K, size=R * T).astype(np.int32)
    off = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = default_initial_params(N, K)
    out = {}
    for mode in a.modes.split(","):
        eng = BaumWelchEngine(N, K, device=0, rank=0, world_size=1, stat_copies=a.copies)
        eng.set_observations(offsets=off, symbols=sym)
        eng.set_params(pi, A, B)
        eng.reset(0.0, 10 ** 9)
        stats = eng.make_stats_buffer()
        ptr = __import__("ctypes").c_void_p(stats.data_ptr())
        if mode == "peer":  # 1-rank peer all-reduce: estep -> push to itself -> wait + sum -> mstep
            import ctypes
            assert eng._lib.hmmbw_set_rank(eng._ctx, 0, 1) == 0
            eng.set_observations(offsets=off, symbols=sym)
            eng.set_params(pi, A, B)
            eng.reset(0.0, 10 ** 9)
            reg, nb = ctypes.c_void_p(), ctypes.c_int64()
            assert eng._lib.hmmbw_peer_region(eng._ctx, ctypes.byref(reg), ctypes.byref(nb)) == 0
            assert eng._lib.hmmbw_peer_attach(eng._ctx, (ctypes.c_void_p * 1)(reg.value), R) == 0
            assert eng._lib.hmmbw_set_option(eng._ctx, 8, 1) == 0
        if mode == "native":  # 1-rank engine communicator: estep -> ncclAllReduce -> mstep in hmmbw_iterate
            import ctypes
            path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so").encode()
            uid = ctypes.create_string_buffer(128)
            assert eng._lib.hmmbw_set_rank(eng._ctx, 0, 1) == 0
            eng.set_observations(offsets=off, symbols=sym)
            eng.set_params(pi, A, B)
            eng.reset(0.0, 10 ** 9)
            assert eng._lib.hmmbw_comm_unique_id(path, uid) == 0
            assert eng._lib.hmmbw_comm_init(eng._ctx, path, uid, 0, 1, R) == 0

        def it(n):
            if mode in ("single", "native", "peer"):
                eng.enqueue_iterations(n)
                return
            if mode == "split":  # the fused multi-rank kernels with no collective (world 1: identity)
                for _ in range(n):
                    eng.iterate_begin(R)
                    eng.iterate_end()
                return
            for _ in range(n):
                eng._lib.hmmbw_estep(eng._ctx, ptr)
                dist.all_reduce(stats)
                eng._lib.hmmbw_mstep(eng._ctx, ptr, R)
        it(10)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it(a.steps)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[mode] = {"us_per_iter": 1e6 * dt / a.steps, "host_enqueue_us_per_iter": 1e6 * t_host / a.steps,
                     "payload_bytes": eng.comm_payload_bytes() if mode in ("native", "peer") else None}
        eng.close()
    print(json.dumps({"R": R, "copies": a.copies, **out}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
