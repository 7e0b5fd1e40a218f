#!/usr/bin/env python3
"""Baum-Welch throughput benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full EM iteration (E-step kernel over every sequence of the rank, the RCCL all-reduce
of the packed statistics when N > 1, the M-step/convergence kernel) on synthetic sequences already
resident in HBM.  Workload (BASELINE cfg3, per GPU): R=10,000 sequences, T=200, N=8 states, K=256
symbols, the reference's left-to-right topology (hmm_training.py:307-312, generalised to N=8) and
uniform random symbols.  Weak scaling: every rank owns 10,000 sequences.

Prints ONE JSON line (rank 0) with the driver's fields plus:
  roofline     — achieved = algorithmic bytes per E-step launch (B_u = 24T + 16NT + 8
                 per sequence) / the E-step kernel's mean duration from HIP events on its stream;
                 traffic = measured HBM bytes per launch from the committed rocprofv3 PMC summary
                 (profiles/), or null when none matches this config.  For N > 16 (the fp64-MFMA wide
                 path, cfg5) the bound is "mfma": achieved = 8 N^2 T flops per sequence / kernel time
                 against the 78.6 TFLOP/s dense fp64 matrix peak.
  cpu_baseline — the oracle C restatement (oracle/bw_oracle.c, log domain like the reference) timed on
                 one host core over a bounded sample of the same workload (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_MFMA_PEAK_TFS = 78.6  # MI355X dense fp64 matrix peak (vendor spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--R", type=int, default=10_000, help="sequences per GPU")
    p.add_argument("--T", type=int, default=200)
    p.add_argument("--N", type=int, default=8)
    p.add_argument("--K", type=int, default=256)
    p.add_argument("--topology", default="left_to_right", choices=["left_to_right", "dense"])
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--no-kernel-timing", action="store_true", help="skip the HIP events")
    p.add_argument("--timing-every", type=int, default=5, help="time every k-th E-step launch")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo only for tests")
    return p.parse_args()


def init_params(N, K, topology, rng):
    from hmm_training_amd.hmm_training import default_initial_params
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    return pi, A, B


def bytes_per_sequence(T, N):
    return 24 * T + 16 * N * T + 8


def flops_per_sequence(T, N):
    return 8 * N * N * T  # forward + backward + xi, fp64


def workload_name(R, T, N, K):
    if (T, N, K) == (200, 8, 256):
        return "cfg3" if R == 10_000 else ("cfg4" if R == 12_500 else "cfg3-shape")
    if (T, N, K) == (400, 64, 1024):
        return "cfg5" if R == 6_250 else "cfg5-shape"
    return "custom"


def find_traffic(cfg_key):
    """Per-launch HBM bytes of the E-step kernel from a committed PMC summary for this config."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*traffic*.json"), recursive=True)):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if d.get("config_key") == cfg_key and d.get("hbm_bytes_per_launch"):
            best = (float(d["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT))
    return best


def cpu_baseline(N, K, T, topology, budget_s, seed):
    """The oracle (C, log domain, single thread) on a bounded sample of the same workload."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed + 1000)
    pi, A, B = init_params(N, K, topology, rng)

    def run(R):
        sym = rng.integers(0, K, size=R * T).astype(np.int64)
        off = np.arange(R + 1, dtype=np.int64) * T
        t0 = time.perf_counter()
        O.hmm_training(off, sym, N, K, 0.0, 1, pi, A, B)
        return time.perf_counter() - t0

    probe_R = 8
    dt = run(probe_R)
    R = int(max(probe_R, min(200_000, probe_R * budget_s / max(dt, 1e-6))))
    dt = run(R)
    return {"value": R / dt, "unit": "utterances/s/iter", "cores": 1, "kind": "port",
            "sample": f"{R} sequences x 1 EM iteration (T={T}, N={N}, K={K}, {topology}) on the oracle "
                      f"restatement oracle/bw_oracle.c, 1 thread, {dt:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = local_rank % max(torch.cuda.device_count(), 1) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(device)

    from hmm_training_amd.engine import BaumWelchEngine

    R, T, N, K = args.R, args.T, args.N, args.K
    rng = np.random.default_rng(args.seed + 7919 * rank)
    symbols = rng.integers(0, K, size=R * T).astype(np.int32)
    offsets = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = init_params(N, K, args.topology, np.random.default_rng(args.seed))

    eng = BaumWelchEngine(N, K, device=device, topology=args.topology, rank=rank, world_size=world)
    eng.set_observations(offsets=offsets, symbols=symbols, n_seq_global=R * world)
    eng.set_params(pi, A, B)
    assert eng.topology == args.topology
    total_iters = args.warmup + args.steps
    eng.reset(0.0, total_iters + 1)  # epsilon 0: no early stop, every timed step is a full iteration
    stats = eng.make_stats_buffer() if world > 1 else None

    eng.enqueue_iterations(args.warmup, stats)
    torch.cuda.synchronize()
    eng.timing(0 if args.no_kernel_timing else args.timing_every)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.enqueue_iterations(1, stats)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, kern_n = eng.timing(0)
    st, _ = eng.status()
    if st.iterations != total_iters:
        raise RuntimeError(f"expected {total_iters} iterations, engine ran {st.iterations}")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = 1000.0 * elapsed / args.steps
    value = R * world * args.steps / elapsed
    kern_s = kern_ms / max(kern_n, 1) / 1000.0
    bu = bytes_per_sequence(T, N)
    wide = N > 16
    cfg_key = f"R{R}_T{T}_N{N}_K{K}_{args.topology}"
    traffic = find_traffic(cfg_key)
    if wide:  # fp64 MFMA recursions (estep_mfma.hpp): priced against the dense fp64 matrix peak
        achieved = flops_per_sequence(T, N) * R / kern_s / 1e12 if kern_s > 0 else float("nan")
        roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": achieved / FP64_MFMA_PEAK_TFS, "traffic": traffic[0] if traffic else None,
                "kernel": "k_estep_mfma + k_bnum_gather (E-step)", "kernel_ms": kern_s * 1000.0,
                "flops_per_launch_algorithmic": flops_per_sequence(T, N) * R,
                "traffic_source": traffic[1] if traffic else None}
    else:
        achieved = bu * R / kern_s / 1e9 if kern_s > 0 else float("nan")
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic[0] if traffic else None,
                "kernel": "k_estep_small (E-step)", "kernel_ms": kern_s * 1000.0,
                "bytes_per_launch_algorithmic": bu * R,
                "traffic_source": traffic[1] if traffic else None}
    wl = workload_name(R, T, N, K)

    if rank == 0:
        out = {
            "metric": f"Baum-Welch utterances/sec/iter (T={T},N={N},K={K})",
            "value": value,
            "unit": "utterances/s/iter",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform random symbols, seeded); reference-topology random init",
            "config": {"workload": f"{wl} per GPU: R={R} sequences x T={T}, N={N} states, K={K} symbols, "
                                   f"{args.topology} A, one EM iteration per step",
                       "sequences_per_gpu": R, "T": T, "N": N, "K": K, "topology": args.topology,
                       "parallelism": f"dp{world}" if world > 1 else "single",
                       "allreduce": ("rccl (engine communicator, engine stream)" if eng.native_comm else
                                     "torch.distributed") if world > 1 else None},
            "roofline": roof,
            "loglik_last": st.last_log_likelihood,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(N, K, T, args.topology, args.cpu_seconds, args.seed)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
