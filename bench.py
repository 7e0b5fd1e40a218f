#!/usr/bin/env python3
"""Baum-Welch throughput benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full EM iteration (E-step kernel over every sequence of the rank, the RCCL all-reduce
of the packed statistics when N > 1, the M-step/convergence kernel) on synthetic sequences already
resident in HBM.  Workloads:
  N = 1: BASELINE cfg3, R = 10,000 sequences, T = 200, N = 8 states, K = 256 symbols;
  N > 1: BASELINE cfg4 shards, 12,500 sequences per GPU (N = 8 is exactly cfg4's 100,000), weak
         scaling (fixed work per GPU);
  --workload cfg5: 6,250 sequences per GPU, T = 400, N = 64, K = 1024 (the fp64-MFMA wide path).
The reference's left-to-right topology (hmm_training.py:307-312, generalised to N states) and
uniform symbols ('U') by default; --symbols H draws them from a ground-truth left-to-right HMM with
Dirichlet(0.3) emission rows (skewed symbol counts).

--gpus N without a launcher (no WORLD_SIZE in the environment) starts N rank processes itself
(127.0.0.1 rendezvous) before anything touches the GPU, and exits with their status; under a
launcher, --gpus must equal WORLD_SIZE.  --dry-run runs the launcher/rendezvous/timing skeleton
with no GPU work (CPU tests).

Prints ONE JSON line (rank 0) with the driver's fields plus:
  roofline     — SURVEY §8(d) for the dominant launch: algorithmic work over the kernel's launch duration
                 (HIP events on the engine stream) against the bounding resource's peak: bound "hbm",
                 B_u = 24T + 16NT + 8 bytes per sequence vs 8 TB/s on the small kernels (a fixed conversion
                 that charges an alpha_hat round trip the kernels never make, so frac can exceed 1); bound
                 "mfma", 8 N^2 T flops per sequence vs 78.6 TF fp64 on the wide path.  traffic = calibrated
                 PMC HBM bytes per launch (profiles/).  binding = the tightest ceiling the counters measure
                 (roofline_bounds: hbm measured bytes, valu, simd_valu, cu_lds, mfma, simd_mfma; the busiest
                 SIMD and CU counted on the engine's launch map), with the profile's provenance (file,
                 collection time, kernel-source hash, fresh = collected on these kernels).
  cpu_baseline — the oracle C restatement (oracle/bw_oracle.c, log domain like the reference) with
                 OpenMP over utterances on the host cores this process may use, timed on a bounded
                 sample of the same workload (rank 0, N=1 only), with its ratio to the reference's
                 own NumPy path measured in the build container, and the same-host ratio
                 of the two (tests/golden/cpu_same_host.py -> profiles/*/cpu_same_host.json).
  comm         — N > 1: ranks of the RCCL communicator the engine created and the all-reduce
                 microseconds per iteration (HIP events around ncclAllReduce on the engine stream).
  synced       — SURVEY §8(d)'s protocol: median of per-iteration times with the 8-byte convergence
                 read-back after every iteration, and the drop-in train loop's ms per iteration.
"""
from __future__ import annotations

import argparse
import glob
import json
import re
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_MFMA_PEAK_TFS = 78.6  # MI355X dense fp64 matrix peak (vendor spec)
# The reference's own NumPy path at cfg3 shape in the build container (BASELINE.md / SURVEY §6)
REF_UTT_PER_S_1CORE = 9.39
REF_UTT_PER_S_8CORES = 79.98

WORKLOADS = {  # name: (sequences per GPU, T, N, K)
    "cfg3": (10_000, 200, 8, 256),
    "cfg4": (12_500, 200, 8, 256),
    "cfg5": (6_250, 400, 64, 1024),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--prewarm-ms", type=float, default=200.0,
                   help="untimed EM iterations for at least this long before the warm-up steps: the GPU clocks "
                        "ramp up over ~35 ms of load after the set-up (profiles/r5/warmup_ramp.txt)")
    p.add_argument("--trace-region", action="store_true",
                   help="print host timestamps of the timed region (diagnostics, stderr)")
    p.add_argument("--workload", default="auto", choices=["auto", *WORKLOADS],
                   help="auto: cfg3 on one GPU, cfg4 shards (12,500 per GPU) on several")
    p.add_argument("--R", type=int, default=None, help="sequences per GPU (overrides the workload)")
    p.add_argument("--T", type=int, default=None)
    p.add_argument("--N", type=int, default=None)
    p.add_argument("--K", type=int, default=None)
    p.add_argument("--topology", default=None, choices=["left_to_right", "dense"],
                   help="default: left_to_right (dense for cfg5)")
    p.add_argument("--symbols", default="U", choices=["U", "H"], help="U: uniform; H: skewed, from a ground-truth HMM")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    p.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may use")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-synced", action="store_true", help="skip the synced-protocol and drop-in measurements")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--no-kernel-timing", action="store_true", help="skip the HIP events")
    p.add_argument("--timing-batch", type=int, default=20,
                   help="E-step launches timed one by one (HIP events) after the timed region")
    p.add_argument("--deterministic", action="store_true", help="fixed-order reductions (no fp atomics), bitwise reproducible")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo only for tests")
    p.add_argument("--allreduce", default="both", choices=["rccl", "peer", "both"],
                   help="N > 1: the engine's all-reduce; both = time RCCL and the peer all-reduce side by side "
                        "(same engine, same protocol) and report the faster as the headline")
    p.add_argument("--dry-run", action="store_true", help="launcher + rendezvous + timing skeleton, no GPU work")
    return p.parse_args(argv)


def resolve_workload(args, world):
    name = args.workload if args.workload != "auto" else ("cfg3" if world == 1 else "cfg4")
    R, T, N, K = WORKLOADS[name]
    custom = any(v is not None for v in (args.R, args.T, args.N, args.K))
    R = args.R if args.R is not None else R
    T = args.T if args.T is not None else T
    N = args.N if args.N is not None else N
    K = args.K if args.K is not None else K
    topo = args.topology or ("dense" if name == "cfg5" else "left_to_right")
    seed = args.seed if args.seed is not None else {"cfg3": 3, "cfg4": 4, "cfg5": 5}[name]
    if custom:
        name = f"custom ({name} shape overridden)"
    return name, R, T, N, K, topo, seed


def init_params(N, K, topology, rng):
    from hmm_training_amd.hmm_training import default_initial_params
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    return pi, A, B


def synthetic_symbols(R, T, N, K, kind, seed):
    """[R*T] int32 symbols.  U: uniform.  H: a ground-truth left-to-right HMM with N
    states, self-loop 0.9, emission rows ~ Dirichlet(0.3 * 1_K), starting in state 0 — skewed symbol
    counts and gamma statistics, as on real codebook data."""
    rng = np.random.default_rng(seed)
    if kind == "U":
        return rng.integers(0, K, size=R * T).astype(np.int32)
    B = rng.dirichlet(np.full(K, 0.3), size=N)
    cdf = np.cumsum(B, axis=1)
    cdf[:, -1] = 1.0
    state = np.zeros(R, dtype=np.int64)
    out = np.empty((R, T), dtype=np.int32)
    for t in range(T):
        if t:
            state = np.minimum(state + (rng.random(R) < 0.1), N - 1)
        out[:, t] = _sample_rows(cdf, state, rng.random(R))
    return np.minimum(out, K - 1).reshape(-1)


def _sample_rows(cdf, state, u):
    res = np.empty(len(state), dtype=np.int32)
    for s in np.unique(state):
        m = state == s
        res[m] = np.searchsorted(cdf[s], u[m], side="right")
    return res


def bytes_per_sequence(T, N):
    return 24 * T + 16 * N * T + 8


def flops_per_sequence(T, N):
    return 8 * N * N * T  # forward + backward + xi, fp64 (informational figure)


def mfma_flops_issued(T, N):
    return 6 * N * N * T  # what k_estep_mfma issues: forward 2N^2, backward 2N^2, xi 2N^2 per step


def kernel_source_hash() -> str:
    """sha256 (first 16 hex digits) of the engine's kernel sources (hmm_training_amd/csrc/*, include/hmmbw.h):
    the profile summaries record the hash of the tree they were collected on, so a bound read from a profile
    of older kernels shows up as stale in the bench line."""
    import hashlib
    h = hashlib.sha256()
    paths = sorted(glob.glob(os.path.join(ROOT, "hmm_training_amd", "csrc", "*"))) + [os.path.join(ROOT, "include", "hmmbw.h")]
    for p in paths:
        with open(p, "rb") as fh:
            h.update(os.path.basename(p).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def _provenance(d, path):
    """Where a committed profile summary came from: file, collection time and kernel-source hash (fresh =
    collected on the kernel sources of this tree)."""
    src = d.get("kernel_src_sha16")
    return {"source": os.path.relpath(path, ROOT), "collected_utc": d.get("collected_utc"), "kernel_src_sha16": src,
            "fresh": src == kernel_source_hash() if src else None}


def find_traffic(cfg_key):
    """Per-launch HBM bytes of the E-step kernel from a committed PMC summary for this config (the newest
    round's, profiles/rN sorted by round number)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*traffic*.json"), recursive=True), key=_round_key):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if d.get("config_key") == cfg_key and d.get("hbm_bytes_per_launch"):
            best = (float(d["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT), _provenance(d, path))
    return best


def _round_key(path):
    """Sort key of a profiles/rN/... path: by round number, then name."""
    rel = os.path.relpath(path, os.path.join(ROOT, "profiles"))
    head = rel.split(os.sep)[0]
    return (int(head[1:]) if head[:1] == "r" and head[1:].isdigit() else -1, rel)


SIMDS = 1024       # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md chip-level parameters)
VALU_CYCLES = 4    # wave64 fp64 VALU issue: 16 lanes per clock per SIMD (78.6 TF fp64 vector peak)
VALU_CYCLES_32 = 2  # wave64 32-bit VALU issue on a SIMD-32 (MI355X_MICROARCH.md; a lone wave: 4)
CLOCK_MAX_GHZ = 2.4  # MI355X max shader clock: the issue bound at the peak clock is the optimistic one
MFMA_F64_CYCLES = 64  # v_mfma_f64_16x16x4_f64: 2,048 flops per SIMD every 64 cycles (78.6 TF / 1,024 SIMDs / 2.4 GHz)
MFMA_F64_FLOPS = 2 * 16 * 16 * 4


def find_issue(cfg_key):
    """VALU instructions per E-step launch and the loaded clock from a committed SQ summary."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "sq_*.json"), recursive=True), key=_round_key):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        for name, k in d.items():
            if isinstance(k, dict) and k.get("config_key") == cfg_key and k.get("SQ_INSTS_VALU") and "gather" not in name:
                # GRBM_GUI_ACTIVE / 8 / kernel time reads high on dispatches under ~0.3 ms
                # (MI355X_MICROARCH.md, DVFS give-back), so the bound is priced at the max clock
                best = {"valu_insts_per_launch": float(k["SQ_INSTS_VALU"]), "clock_ghz": CLOCK_MAX_GHZ,
                        "valu_fp64_per_launch": k.get("valu_fp64_insts"),
                        "mfma_busy_cycles": k.get("SQ_VALU_MFMA_BUSY_CYCLES"),
                        "lds_array_cycles": k.get("SQ_LDS_IDX_ACTIVE"),
                        "lds_insts": k.get("SQ_INSTS_LDS"),
                        "waves_counted": k.get("SQ_WAVES"),
                        "clock_ghz_grbm_estimate": k.get("clock_ghz"), "source": os.path.relpath(path, ROOT),
                        "provenance": _provenance(k, path)}
    return best


CUS = SIMDS // 4


def _newest_json(pattern, accept):
    """The newest round's committed profile (profiles/rN/...) matching `pattern` whose content passes accept."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", pattern), recursive=True), key=_round_key):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if accept(d):
            best = (d, path)
    return best


def find_chain():
    """Measured dependent-chain cycles per step (tools/ubench_chain.hip, profiles/rN/ubench_chain.txt): the
    forward step (DPP shift || multiply -> fma) and the backward beta step (multiply -> DPP shift -> fma), one
    wave per SIMD and two."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "ubench_chain.txt"), recursive=True), key=_round_key):
        d, src = {}, None
        with open(path) as fh:
            for line in fh:
                m = re.match(r"#\s*kernel_src_sha16\s+(\w+)", line)
                if m:
                    src = m.group(1)
                m = re.match(r"(.+?)\s+waves\s+(\d+)\s+([\d.]+) cycles/step", line)
                if m:
                    d[(m.group(1).strip(), int(m.group(2)))] = float(m.group(3))
        f1, b1 = d.get(("forward step (dpp+mul+fma)", 4)), d.get(("backward beta step (mul+dpp+fma)", 4))
        if f1 and b1:
            best = {"forward": f1, "backward": b1, "forward_2waves": d.get(("forward step (dpp+mul+fma)", 8)),
                    "backward_2waves": d.get(("backward beta step (mul+dpp+fma)", 8)),
                    "source": os.path.relpath(path, ROOT),
                    "provenance": {"source": os.path.relpath(path, ROOT), "kernel_src_sha16": src,
                                   "fresh": None, "note": "a microbenchmark of the step's instruction chain"}}
    return best


def roofline_latency(R, T, N, topo, kern_s, issue, lmap):
    """Left-to-right headline (N <= 8 LDS tables): the dependent-chain bound and a per-phase model of the busiest
    SIMD, read from committed profiles of the newest round:
      phases   profiles/rN/phase_lr_*.json (tools/phase_times.py --json): the prologue (kernel start -> LDS tables
               written) and the tail (backward done -> statistics flushed) of the waves on two-wave SIMDs, measured;
      chain    profiles/rN/ubench_chain.txt: cycles per dependent forward / backward step;
      isa      profiles/rN/isa_lr_steps.json (tools/isa_steps.py): instructions per step of the steady loops.
    latency      = prologue + T x (chain_fwd + chain_bwd) / clock + tail: no schedule can beat the chains.
    phase_model  = prologue + T x (max over {chain, busiest-SIMD VALU pipe, single-wave issue, busiest-CU LDS}
                   per step, forward and backward) / clock + tail; its frac is the share of the kernel time that
                   the chains, the VALU and the LDS jointly explain; the rest (`unexplained_us`) is itemised."""
    if N > 8 or topo != "left_to_right" or kern_s <= 0:
        return {}
    ph = _newest_json("phase_lr_*.json", lambda d: d.get("T") == T and d.get("N") == N and d.get("R") == R
                      and d.get("topology") == topo and "busy" in d.get("classes", {}))
    isa = _newest_json("isa_lr_steps.json", lambda d: "forward" in d.get("loops", {}))
    ch = find_chain()
    if not (ph and isa and ch):
        return {}
    phd, php = ph
    busy = phd["classes"]["busy"]
    pro = busy["at_tables_us"]["p50"]
    tail = busy["at_flush_us"]["p50"] - busy["at_backward_us"]["p50"]
    f = CLOCK_MAX_GHZ * 1e3  # cycles per us
    out = {}
    lat = pro + T * (ch["forward"] + ch["backward"]) / f + tail
    out["latency"] = {"achieved": lat / (kern_s * 1e6), "peak": 1.0, "unit": "fraction of the kernel time",
                      "frac": lat / (kern_s * 1e6), "t_bound_us": lat,
                      "parts_us": {"prologue": pro, "forward_chain": T * ch["forward"] / f,
                                   "backward_chain": T * ch["backward"] / f, "tail": tail},
                      "chain_cycles_per_step": {"forward": ch["forward"], "backward": ch["backward"]},
                      "source": [os.path.relpath(php, ROOT), ch["source"]],
                      "provenance": _provenance(phd, php)}
    wmax = 2
    wcu = engine_waves(R, N, lmap)[2] if lmap else 6
    lds_cyc = (issue["lds_array_cycles"] / issue["lds_insts"]) if issue and issue.get("lds_insts") else 8.0
    parts, steps = {}, {}
    for nm in ("forward", "backward"):
        c = isa[0]["loops"][nm]["per_step"]
        n_all = sum(v for k, v in c.items() if k not in ("dpp", "lds_atomic"))
        simd = wmax * (VALU_CYCLES * c.get("f64", 0) + VALU_CYCLES_32 * c.get("v32", 0))
        single = 4.0 * n_all
        lds = wcu * c.get("lds", 0) * lds_cyc
        step = {"chain": ch[nm], "simd_valu_pipe": simd, "single_wave_issue": single, "cu_lds": lds}
        steps[nm] = {**{k: round(v, 2) for k, v in step.items()}, "binding": max(step, key=step.get),
                     "measured_busy": 1e3 * busy[("tables->forward_us" if nm == "forward" else "forward->backward_us")]["p50"]
                     * CLOCK_MAX_GHZ / T}
        parts[nm] = T * max(step.values()) / f
    model = pro + parts["forward"] + parts["backward"] + tail
    meas_end = busy["at_flush_us"]["p50"]
    out["phase_model"] = {"achieved": model / (kern_s * 1e6), "peak": 1.0,
                          "unit": "fraction of the kernel time the per-phase bounds explain", "frac": model / (kern_s * 1e6),
                          "t_bound_us": model, "parts_us": {"prologue": pro, **parts, "tail": tail},
                          "cycles_per_step": steps, "waves_on_busiest_simd": wmax, "waves_on_busiest_cu": wcu,
                          "lds_cycles_per_instruction": lds_cyc,
                          "unexplained_us": {"forward": busy["tables->forward_us"]["p50"] - parts["forward"],
                                             "backward": busy["forward->backward_us"]["p50"] - parts["backward"],
                                             "phase_build_span_vs_kernel": kern_s * 1e6 - meas_end},
                          "source": [os.path.relpath(php, ROOT), os.path.relpath(isa[1], ROOT), ch["source"]],
                          "provenance": _provenance(phd, php), "isa_provenance": _provenance(isa[0], isa[1])}
    return out


def engine_waves(R, N, lmap=None):
    """(active waves, waves on the busiest SIMD, waves on the busiest CU) of one E-step launch.

    With the engine's launch map (BaumWelchEngine.launch_map, HMMBW_INFO_*: the spread map of the small
    kernels puts one full 4-wave workgroup on every CU, then the waves past one per SIMD into workgroups of
    `extra_waves` active waves) the busiest CU and SIMD are counted on that map, workgroup i placed on CU
    i mod 256 (dispatch order; the kernels admit two workgroups per CU) and a CU's waves spread over its 4
    SIMDs.  Without it (CPU tests): small kernels 64 / G sequences per wave, wide tiles of 16 sequences
    with NP / 16 waves, and the pigeonhole minimum ceil(waves / 1,024) per SIMD, ceil(waves / 256) per CU."""
    if lmap and lmap.get("waves") and not lmap.get("work_queue"):
        waves, nwg, wpw = lmap["waves"], lmap["workgroups"], lmap["waves_per_workgroup"]
        full, extra = min(lmap["full_workgroups"], nwg), lmap["extra_waves"] or wpw
        cu = [0] * CUS
        left = waves
        for i in range(nwg):
            w = min(wpw if i < full else extra, left)
            left -= w
            cu[i % CUS] += w
        wcu = max(cu)
        return waves, -(-wcu // 4), wcu
    if N <= 16:
        G = 2 if N <= 2 else 4 if N <= 4 else 8 if N <= 8 else 16
        waves = -(-R // (64 // G))
    else:
        waves = -(-R // 16) * (-(-N // 16))
    return waves, -(-waves // SIMDS), -(-waves // CUS)


OPT_ALLREDUCE_KEY = 8  # HMMBW_OPT_ALLREDUCE (include/hmmbw.h): 0 = RCCL / the caller's all-reduce, 1 = peer


def torch_allreduce_iteration(eng, dist, device, backend):
    """One EM iteration through the split ABI with torch.distributed's all-reduce of the statistics in
    between (hmmbw_iterate_begin -> dist.all_reduce -> hmmbw_iterate_end): the reference path of bench's leg
    check.  The buffer goes through a torch tensor (device memory for nccl, host for gloo) by hipMemcpy."""
    import ctypes
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    ptr, n = eng.iterate_begin()
    torch.cuda.synchronize()
    if backend == "nccl":
        t = torch.empty(n, dtype=torch.float64, device=f"cuda:{device}")
        assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), 8 * n, 3) == 0
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(t.data_ptr()), 8 * n, 3) == 0
    else:
        h = np.empty(n, dtype=np.float64)
        assert hip.hipMemcpy(h.ctypes.data, ctypes.c_void_p(ptr), 8 * n, 2) == 0
        t = torch.from_numpy(h)
        dist.all_reduce(t)
        assert hip.hipMemcpy(ctypes.c_void_p(ptr), h.ctypes.data, 8 * n, 1) == 0
    torch.cuda.synchronize()
    eng.iterate_end()


def roofline_bounds(R, T, N, kern_s, traffic, issue, estep_s=None, lmap=None, topo=None):
    """Every ceiling that applies to the dominant launch, each as achieved / peak of ONE resource, so every
    frac is <= 1 when the measurement and the model are right; the binding bound is the largest frac.

    hbm        measured HBM bytes per launch (calibrated PMC FETCH/WRITE, profiles/) / kernel time vs 8 TB/s.
    valu       all VALU instructions of the launch (SQ_INSTS_VALU) spread evenly over the 1,024 SIMDs at the
               2.4 GHz max clock: on a SIMD-32 a wave64 fp64 add / mul / fma / transcendental takes 4 cycles
               (half the fp32 rate), every other VALU instruction 2 (MI355X_MICROARCH.md, SIMD-32), with the
               fp64 share from the SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 counters.
    simd_valu  the busiest SIMD: it runs w waves (the launch map's busiest SIMD, engine_waves) and must issue
               all their VALU instructions on its one VALU pipe, max(w x (4 n64 + 2 (n - n64)), 4 n) cycles
               for n VALU instructions per wave of which n64 fp64 (a single wave issues at most every 4
               cycles); achieved / peak = that time / the kernel time, written as an issue rate.
    cu_lds     the busiest CU's LDS array (shared by its 4 SIMDs): its waves x the LDS-array cycles per wave
               (SQ_LDS_IDX_ACTIVE, bank-conflict cycles included) at the max clock / the kernel time.
    mfma, simd_mfma  (wide path) the same for the fp64 matrix pipe: every wave issues 48 dependent-block
               v_mfma_f64_16x16x4 per step (forward 4NT, backward 4NT, xi 4NT at NT = 4), 64 cycles each.
    """
    waves, wmax, wcu = engine_waves(R, N, lmap)
    t_clock = CLOCK_MAX_GHZ * 1e9
    out = {"waves_per_launch": waves, "waves_on_busiest_simd": wmax, "waves_on_busiest_cu": wcu,
           "wave_map": ("engine launch map (HMMBW_INFO_*), workgroup i on CU i mod 256"
                        + (" (joined: extra workgroup i runs as waves 4.. of workgroup i, the same CU)" if lmap.get("joined") else "")
                        if lmap and not lmap.get("work_queue") else "pigeonhole (no launch map)"),
           "clock_ghz": CLOCK_MAX_GHZ}
    if traffic and kern_s > 0:
        ach = traffic[0] / kern_s / 1e9
        out["hbm"] = {"achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                      "bytes_per_launch": traffic[0], "source": traffic[1], "provenance": traffic[2]}
    if N > 16:
        nt = -(-N // 16)
        mfma_wave = 3 * 4 * nt * T  # per step: forward 4NT, backward 4NT, xi NT x 4 (estep_mfma.hpp)
        t_e = estep_s if estep_s else kern_s
        peak_simd = t_clock / MFMA_F64_CYCLES * MFMA_F64_FLOPS / 1e12  # TFLOP/s of one SIMD's matrix pipe
        ach_bal = waves * mfma_wave * MFMA_F64_FLOPS / t_e / 1e12
        out["mfma"] = {"achieved": ach_bal, "peak": peak_simd * SIMDS, "unit": "TFLOP/s",
                       "frac": ach_bal / (peak_simd * SIMDS), "mfma_per_wave": mfma_wave,
                       "kernel": "k_estep_mfma", "kernel_ms": 1e3 * t_e}
        ach_s = wmax * mfma_wave * MFMA_F64_FLOPS / t_e / 1e12
        out["simd_mfma"] = {"achieved": ach_s, "peak": peak_simd, "unit": "TFLOP/s per SIMD",
                            "frac": ach_s / peak_simd, "mfma_per_wave": mfma_wave,
                            "t_bound_us": 1e6 * wmax * mfma_wave * MFMA_F64_CYCLES / t_clock,
                            "kernel": "k_estep_mfma", "kernel_ms": 1e3 * t_e}
    if issue and kern_s > 0 and N <= 16 and issue.get("valu_fp64_per_launch") is not None:
        n_all = issue["valu_insts_per_launch"]
        n64 = issue["valu_fp64_per_launch"]
        cyc_all = VALU_CYCLES * n64 + VALU_CYCLES_32 * (n_all - n64)  # SIMD-cycles of the whole launch
        t_bal = cyc_all / SIMDS / t_clock
        out["valu"] = {"achieved": t_bal / kern_s, "peak": 1.0, "unit": "fraction of SIMD VALU issue cycles (mean)",
                       "frac": t_bal / kern_s, "t_bound_us": 1e6 * t_bal, "valu_per_launch": n_all,
                       "valu_fp64_per_launch": n64, "source": issue["source"], "provenance": issue["provenance"]}
        nw, n64w = n_all / waves, n64 / waves
        cyc_simd = max(wmax * (VALU_CYCLES * n64w + VALU_CYCLES_32 * (nw - n64w)), VALU_CYCLES * nw)
        t_simd = cyc_simd / t_clock
        out["simd_valu"] = {"achieved": t_simd / kern_s, "peak": 1.0,
                            "unit": "fraction of the busiest SIMD's VALU issue cycles", "frac": t_simd / kern_s,
                            "t_bound_us": 1e6 * t_simd, "valu_per_wave": nw, "valu_fp64_per_wave": n64w,
                            "waves_on_busiest_simd": wmax, "source": issue["source"], "provenance": issue["provenance"]}
        if lmap and lmap.get("split_extra"):
            # The map counts sequence-group waves.  A split group runs on two waves (A: forward + upper backward,
            # B: beta pre-sweep + lower backward), each on its own SIMD, so the busiest SIMD's second wave holds
            # only part of a group: charging it a whole group makes this an upper bound on that SIMD's load.
            out["simd_valu"]["note"] = "upper bound: a split extra group's A or B wave charged as a whole group"
            out["split_extra_groups"] = waves - min(lmap["full_workgroups"], lmap["workgroups"]) * lmap["waves_per_workgroup"]
    if issue and kern_s > 0 and N <= 16 and issue.get("lds_array_cycles"):
        # SQ_LDS_IDX_ACTIVE = every LDS-array cycle of the launch, bank-conflict cycles included, per active wave
        t_lds = wcu * issue["lds_array_cycles"] / waves / t_clock
        out["cu_lds"] = {"achieved": t_lds / kern_s, "peak": 1.0, "unit": "fraction of the busiest CU's LDS-array cycles",
                         "frac": t_lds / kern_s, "t_bound_us": 1e6 * t_lds, "waves_on_busiest_cu": wcu,
                         "lds_cycles_per_wave": issue["lds_array_cycles"] / waves, "source": issue["source"],
                         "provenance": issue["provenance"]}
    if topo is not None:
        out.update(roofline_latency(R, T, N, topo, kern_s, issue, lmap))
    cands = {k: v for k, v in out.items() if isinstance(v, dict) and "frac" in v}
    out["binding"] = max(cands, key=lambda k: cands[k]["frac"]) if cands else None
    return out


def host_threads(requested=0):
    if requested > 0:
        return requested
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(N, K, T, topology, budget_s, seed, symbols="U", threads=0):
    """The oracle (C, log domain, OpenMP over utterances) on a bounded sample of the same workload."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed + 1000)
    pi, A, B = init_params(N, K, topology, rng)
    nth = O.set_threads(host_threads(threads))

    def run(R):
        sym = synthetic_symbols(R, T, N, K, symbols, seed + 1000 + R).astype(np.int64)
        off = np.arange(R + 1, dtype=np.int64) * T
        t0 = time.perf_counter()
        O.hmm_training(off, sym, N, K, 0.0, 1, pi, A, B)
        return time.perf_counter() - t0

    try:
        probe_R = 8 * nth
        dt = run(probe_R)
        # batches of at most 200,000 sequences (bounded host memory) until the time budget is spent
        batch = int(max(probe_R, min(200_000, probe_R * budget_s / max(dt, 1e-6))))
        R, dt = 0, 0.0
        while dt < budget_s and R < 5_000_000:
            dt += run(batch)
            R += batch
    finally:
        O.set_threads(1)
    value = R / dt
    out = {"value": value, "unit": "utterances/s/iter", "cores": nth, "kind": "port",
           "cpu_model": cpu_model(), "nproc_visible": os.cpu_count(),
           "sample": f"{R} sequences x 1 EM iteration (T={T}, N={N}, K={K}, {topology}, symbols {symbols}) on the "
                     f"oracle restatement oracle/bw_oracle.c, OpenMP over utterances on {nth} threads, {dt:.1f} s",
           "ratio_vs_reference_8cores": value / REF_UTT_PER_S_8CORES,
           "ratio_per_core_vs_reference": (value / nth) / REF_UTT_PER_S_1CORE,
           "reference_note": "reference NumPy path (HMM/hmm_training.py) measured in the build container at cfg3 "
                             "shape: 9.39 utt/s/iter on 1 core, 79.98 on 8 (BASELINE.md); different host"}
    same = find_same_host()
    if same and (T, N, K) == (200, 8, 256):
        # the reference and the oracle timed back to back on ONE host (tests/golden/cpu_same_host.py): the
        # oracle's per-core speed-up over the reference there, and what it implies for the reference on
        # this box's cores (the reference itself cannot run here)
        r = same["ratio_oracle_vs_reference_per_core"]
        out["same_host"] = {"host": same["host"], "source": same["source"],
                            "reference_utt_per_s_1core": same["reference_utt_per_s_1core"],
                            "oracle_utt_per_s_1thread": same["oracle_utt_per_s_1thread"],
                            "ratio_oracle_vs_reference_per_core": r,
                            "reference_estimate_here_utt_per_s": value / r,
                            "note": "reference_estimate_here = this box's oracle rate on "
                                    f"{nth} threads / the same-host per-core ratio (assumes the reference, "
                                    "single-threaded NumPy, would scale over processes as the oracle over threads)"}
    return out


def find_same_host():
    """The latest committed same-host timing of the reference vs the oracle (profiles/*/cpu_same_host.json)."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "cpu_same_host.json")))
    if not paths:
        return None
    try:
        with open(paths[-1]) as fh:
            d = json.load(fh)
    except Exception:
        return None
    d["source"] = os.path.relpath(paths[-1], ROOT)
    return d


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv):
    """--gpus N without a launcher: start N rank processes (one per GPU) before any GPU call."""
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:  # one rank failed: the others would wait forever in a collective
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc if rc >= 0 else 128 - rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch(args, argv)
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    wl, R, T, N, K, topo, seed = resolve_workload(args, world)

    import torch
    import torch.distributed as dist

    if args.dry_run:
        return dry_run(args, world, rank, wl, R, T, N, K, topo)

    device = local_rank % max(torch.cuda.device_count(), 1) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(device)

    from hmm_training_amd.engine import BaumWelchEngine

    symbols = synthetic_symbols(R, T, N, K, args.symbols, seed + 7919 * rank)
    offsets = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = init_params(N, K, topo, np.random.default_rng(seed))

    # peer waits give up after 5 s (ranks enter each leg together after a barrier; a failed leg is dropped)
    eng = BaumWelchEngine(N, K, device=device, topology=topo, rank=rank, world_size=world,
                          deterministic=args.deterministic, allreduce=args.allreduce, peer_timeout_ms=5000)
    t_up = time.perf_counter()
    eng.set_observations(offsets=offsets, symbols=symbols, n_seq_global=R * world)
    eng.set_params(pi, A, B)
    torch.cuda.synchronize()
    upload_s = time.perf_counter() - t_up
    assert eng.topology == topo
    eng.reset(0.0, 1 << 40)  # epsilon 0: no early stop, every timed step is a full iteration
    stats = eng.make_stats_buffer() if world > 1 and not eng.native_comm else None
    n_iter = [0]

    def enqueue(n):
        eng.enqueue_iterations(n, stats)
        n_iter[0] += n

    def prewarm(ms):
        """Untimed iterations for about `ms` of GPU work: one batch of 20 measures the iteration time, then
        every rank enqueues the same count (the largest over ranks: each iteration is a collective)."""
        if ms <= 0:
            return
        t_start = time.perf_counter()
        enqueue(20)
        torch.cuda.synchronize()
        per = max((time.perf_counter() - t_start) / 20, 1e-6)
        n = min(int(ms / 1000.0 / per), 200_000)
        if world > 1:
            t = torch.tensor([n], dtype=torch.int64, device=f"cuda:{device}" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            n = int(t.item())
        if n > 20:
            enqueue(n - 20)
        torch.cuda.synchronize()

    def leg(steps, warmup):
        """Warm-up, then EXACTLY `steps` EM iterations between barrier + synchronize brackets (max over
        ranks), then the per-launch timing batch (HIP events) outside the timed region."""
        enqueue(warmup)
        torch.cuda.synchronize()
        eng.timing(0)
        eng.comm_info(reset=True)
        # The engine launches on torch's current stream (BaumWelchEngine binds it), so one event pair on
        # that stream around the whole timed region gives the GPU time per step without perturbing it.
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()  # the HIP events are created at their first record (~30 us of host time): not in the region
        ev1.record()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        t_ev0 = time.perf_counter()
        enqueue(steps)  # one hmmbw_iterate(steps): the host enqueues the K launches back to back
        t_enq = time.perf_counter()
        ev1.record()
        torch.cuda.synchronize()
        t_sync = time.perf_counter()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if args.trace_region:
            print(f"[trace rank {rank}] ev0.record {1e6 * (t_ev0 - t0):.1f} us, enqueue({steps}) "
                  f"{1e6 * (t_enq - t_ev0):.1f} us, ev1.record + sync {1e6 * (t_sync - t_enq):.1f} us, "
                  f"region {1e6 * elapsed:.1f} us, GPU {1e3 * ev0.elapsed_time(ev1):.1f} us", file=sys.stderr, flush=True)
        r = {"gpu_ms_step": ev0.elapsed_time(ev1) / steps, "kern_ms": 0.0, "kern_n": 0, "est_ms": 0.0, "est_n": 0,
             "ar_ms": 0.0, "ar_n": 0}
        # a device-side failure (a peer all-reduce timeout) is recorded, not raised, until every rank has
        # passed the collective below: no rank may leave the leg while the others wait in it
        try:
            st, _ = eng.status()
            r["error"] = None if st.iterations == n_iter[0] else \
                f"expected {n_iter[0]} iterations, engine ran {st.iterations}"
        except Exception as e:  # noqa: BLE001 - reported in the JSON line, or raised for the first leg
            r["error"] = str(e)
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64,
                             device=f"cuda:{device}" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        r["elapsed"] = elapsed
        r["comm_ranks"] = eng.comm_info()[0]
        # E-step launches timed one by one (event pairs around each launch serialise the queue, so this
        # reads ~1-2 us above the undisturbed kernel), in a separate batch after the timed region; plus the
        # all-reduce per iteration on the engine's own path
        if world > 1:  # every rank learns whether any rank failed
            ok = torch.tensor([0 if r["error"] else 1], dtype=torch.int32,
                              device=f"cuda:{device}" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and not r["error"]:
                r["error"] = "another rank failed this leg"
        if r["error"]:
            r["allreduce"] = eng.allreduce
            return r
        if not args.no_kernel_timing:
            eng.timing(1)
            eng.comm_info(reset=True)
            enqueue(args.timing_batch)
            torch.cuda.synchronize()
            r["est_ms"], r["est_n"] = eng.timing_split()  # wide path: the E-step kernel alone (before the gather)
            r["kern_ms"], r["kern_n"] = eng.timing(0)
            r["comm_ranks"], r["ar_ms"], r["ar_n"] = eng.comm_info(reset=True)
        r["allreduce"] = eng.allreduce
        return r

    legs, failed = {}, {}
    prewarm(args.prewarm_ms)
    first = leg(args.steps, args.warmup)
    if first["error"]:
        raise RuntimeError(first["error"])
    legs[first["allreduce"] or "none"] = first
    if world > 1 and args.allreduce == "both" and eng._rccl_ok and eng._peer_ok:
        # the other all-reduce on the same engine and data, same protocol: both are measured side by side
        other = "peer" if first["allreduce"] == "rccl" else "rccl"
        eng.set_allreduce(other)
        r2 = leg(args.steps, max(2, min(args.warmup, 10)))
        if r2["error"]:
            # the line still reports the first leg; the engine restarts from a clean state on it
            failed[other] = r2["error"]
            eng.set_allreduce(first["allreduce"])
            eng.reset(0.0, 1 << 40)
            n_iter[0] = 0
        else:
            legs[other] = r2
    agree = None
    ref_kind = None
    if world > 1 and any(k in ("rccl", "peer") for k in legs):
        # every engine all-reduce must give the same EM run as a reference before it is a headline: the same
        # few iterations from the same parameters on each, L traces (hmm_training.py:503) compared at rtol
        # 1e-9.  The reference is the RCCL leg when it ran, else the torch.distributed path (the split ABI
        # with dist.all_reduce of the statistics in between).  A leg that disagrees (e.g. a peer exchange that
        # is not coherent over xGMI) is dropped on every rank; if none is left, the torch path is timed.
        def trace_of(kind):
            eng.set_params(pi, A, B)
            try:
                if kind == "torch":
                    eng.set_option(OPT_ALLREDUCE_KEY, 0)  # the caller's all-reduce (no peer push)
                    eng.reset(0.0, 3)
                    for _ in range(3):
                        torch_allreduce_iteration(eng, dist, device, args.dist_backend)
                else:
                    eng.set_allreduce(kind)
                    eng.reset(0.0, 3)
                    eng.enqueue_iterations(3, stats)
                return [L for L, _ in eng.status(0, 3)[1]]
            except Exception as e:  # noqa: BLE001 - a device-side failure of the check drops that leg
                return str(e)
        ref_kind = "rccl" if "rccl" in legs else "torch"
        traces = {k: trace_of(k) for k in legs if k in ("rccl", "peer")}
        if ref_kind == "torch":
            traces["torch"] = trace_of("torch")
        ref_t = traces.get(ref_kind)
        agree = {}
        for kind, tr in traces.items():
            ok = isinstance(tr, list) and isinstance(ref_t, list) and np.allclose(tr, ref_t, rtol=1e-9, atol=0.0)
            agree[kind] = bool(ok)
            if kind in legs and kind != ref_kind and not ok:
                failed[kind] = f"L trace differs from the {ref_kind} reference's: {tr} vs {ref_t}"
                legs.pop(kind)
        # every rank drops the same legs
        keep = torch.tensor([1 if k in legs else 0 for k in ("rccl", "peer")], dtype=torch.int32,
                            device=f"cuda:{device}" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(keep, op=dist.ReduceOp.MIN)
        for i, k in enumerate(("rccl", "peer")):
            if k in legs and int(keep[i]) == 0:
                legs.pop(k)
                failed.setdefault(k, "another rank's check failed")
        if "rccl" in legs or "peer" in legs:
            eng.set_allreduce(next(k for k in ("rccl", "peer") if k in legs))
        n_iter[0] = 0
        if not legs:  # every engine leg dropped: time the torch.distributed path instead (a valid line)
            eng.set_option(OPT_ALLREDUCE_KEY, 0)
            eng._native = False
            stats = eng.make_stats_buffer()
            eng.reset(0.0, 1 << 40)
            r3 = leg(args.steps, max(2, min(args.warmup, 10)))
            if r3["error"]:
                raise RuntimeError("every all-reduce leg failed: " + json.dumps(failed) + "; torch: " + r3["error"])
            r3["allreduce"] = None
            legs["torch"] = r3
        else:
            eng.reset(0.0, 1 << 40)
    # the headline is the faster leg (both run the full EM iteration; config.allreduce names it)
    best = max(legs, key=lambda k: -legs[k]["elapsed"])
    L = legs[best]
    eng.set_allreduce(best) if best in ("rccl", "peer") and len(legs) > 1 else None
    elapsed, gpu_ms_step = L["elapsed"], L["gpu_ms_step"]
    kern_ms, kern_n, est_ms, est_n = L["kern_ms"], L["kern_n"], L["est_ms"], L["est_n"]
    ar_ms, ar_n, comm_ranks = L["ar_ms"], L["ar_n"], L["comm_ranks"]
    st, _ = eng.status()

    synced = None
    if not args.no_synced:
        synced = synced_protocol(eng, stats, world, dist, R)

    ms_step = 1000.0 * elapsed / args.steps
    value = R * world * args.steps / elapsed
    # the kernel time the roofline uses: single rank on the small kernels, every step is ONE launch
    # (E-step with the merged M-step), so the GPU time per step over the timed region IS the launch
    # duration (+ the ~1 us dispatch gap between back-to-back launches: conservative); elsewhere (the
    # wide path's three launches, the all-reduce of N > 1) the per-launch event batch above
    single_kernel = world == 1 and N <= 16 and not args.deterministic
    if single_kernel or kern_n == 0:
        kern_s, kern_src = gpu_ms_step / 1000.0, "HIP events around the timed region / steps (one launch per step)"
    else:
        kern_s, kern_src = kern_ms / kern_n / 1000.0, f"HIP events around each of {kern_n} E-step launches after the timed region"
    bu = bytes_per_sequence(T, N)
    wide = N > 16
    cfg_key = f"R{R}_T{T}_N{N}_K{K}_{topo}" + ("_H" if args.symbols == "H" else "")
    traffic = find_traffic(cfg_key)
    issue = find_issue(cfg_key)
    estep_s = (est_ms / est_n / 1000.0) if est_n else None
    lmap = eng.launch_map()
    small_kernel = "k_estep_join" if lmap.get("joined") else "k_estep_small"  # the joined map's 8-wave kernel
    bounds = roofline_bounds(R, T, N, kern_s, traffic, issue, estep_s, lmap, topo)
    # The roofline (the task's contract and SURVEY §8(d)): ALGORITHMIC work per launch over the kernel's
    # average launch duration against the peak of the bounding resource.  Small kernels: HBM, B_u = 24T +
    # 16NT + 8 bytes per sequence (a fixed conversion: it charges an alpha_hat round trip the
    # checkpoint-and-recompute kernels never make, so frac can exceed 1).  Wide path: the fp64 matrix
    # pipe, 8 N^2 T flops per sequence over the E-step kernel.  `binding` is the tightest ceiling the
    # counters measure (largest achieved / peak among `bounds`, each <= 1 when measurement and model are
    # right), with the profile it came from and whether that profile was collected on these kernels.
    b = bounds.get(bounds.get("binding") or "", None)
    if wide:
        t_e = estep_s if estep_s else kern_s
        ach = flops_per_sequence(T, N) * R / t_e / 1e12 if t_e > 0 else float("nan")
        model = {"bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                 "frac": ach / FP64_MFMA_PEAK_TFS, "units_per_launch": R,
                 "work_per_unit": f"{flops_per_sequence(T, N)} flops (SURVEY §8(d): 8 N^2 T per sequence)",
                 "issued_frac_6N2T": mfma_flops_issued(T, N) * R / t_e / 1e12 / FP64_MFMA_PEAK_TFS,
                 "kernel": "k_estep_mfma", "kernel_ms": 1e3 * t_e}
    else:
        ach = bu * R / kern_s / 1e9 if kern_s > 0 else float("nan")
        model = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                 "units_per_launch": R,
                 "work_per_unit": f"{bu} bytes (SURVEY §8(d): 24 T + 16 N T + 8 per sequence)",
                 "kernel": small_kernel, "kernel_ms": 1e3 * kern_s}
    roof = {"bound": model["bound"], "achieved": model["achieved"], "peak": model["peak"], "unit": model["unit"],
            "frac": model["frac"], "traffic": traffic[0] if traffic else None,
            "model": model,
            "kernel": "k_estep_mfma + k_bnum_gather (E-step)" if wide else f"{small_kernel} (E-step)",
            "kernel_ms": kern_s * 1000.0, "kernel_time_source": kern_src,
            "binding": ({"resource": bounds["binding"], **{k: b[k] for k in ("achieved", "peak", "unit", "frac")},
                         "t_bound_us": b.get("t_bound_us"), "provenance": b.get("provenance")} if b else None),
            "hbm_frac_measured": bounds["hbm"]["frac"] if "hbm" in bounds else None,
            "traffic_provenance": traffic[2] if traffic else None,
            "kernel_src_sha16": kernel_source_hash(),
            "bounds": bounds, "launch_map": lmap,
            "gpu_ms_per_step": gpu_ms_step,
            "kernel_ms_per_launch_events": kern_ms / kern_n if kern_n else None}

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
            "data": f"synthetic ({'uniform' if args.symbols == 'U' else 'HMM-generated skewed'} symbols, seeded); "
                    "reference-topology init",
            "config": {"workload": f"{wl}: R={R} sequences per GPU ({R * world} total) x T={T}, N={N} states, "
                                   f"K={K} symbols, {topo} A, symbols {args.symbols}, one EM iteration per step",
                       "sequences_per_gpu": R, "sequences_total": R * world, "T": T, "N": N, "K": K,
                       "topology": topo, "symbols": args.symbols, "deterministic": bool(args.deterministic),
                       "parallelism": f"dp{world}" if world > 1 else "single",
                       "allreduce": ({"rccl": "rccl (engine communicator, engine stream)",
                                      "peer": "peer (engine push / wait + sum over IPC-mapped regions, engine stream)"}
                                     .get(best, f"torch.distributed ({args.dist_backend})")) if world > 1 else None},
            "roofline": roof,
            "comm": {"kind": best, "rccl_comm_ranks": comm_ranks,
                     "allreduce_us_per_iter": 1000.0 * ar_ms / ar_n if ar_n else None,
                     "allreduce_timed": ar_n,
                     "payload_bytes": eng.comm_payload_bytes() if eng.native_comm else 8 * eng.stats_len,
                     "legs": {k: {"value": R * world * args.steps / v["elapsed"],
                                  "ms_per_step": 1000.0 * v["elapsed"] / args.steps,
                                  "allreduce_us_per_iter": 1000.0 * v["ar_ms"] / v["ar_n"] if v["ar_n"] else None,
                                  "kernel_ms_per_launch_events": v["kern_ms"] / v["kern_n"] if v["kern_n"] else None}
                              for k, v in legs.items()},
                     "legs_failed": failed, "legs_agree": agree, "legs_reference": ref_kind,
                     "legs_detail": {k: {"payload_bytes": eng.comm_payload_bytes() if eng.native_comm else 8 * eng.stats_len,
                                         "peer_chunks": eng.peer_chunks() if k == "peer" else None,
                                         "peer_flags_written_and_polled_per_rank_per_iter": (
                                             world * eng.peer_chunks() if k == "peer" else None),
                                         "collectives_per_iter": 1}
                                     for k in legs}}
            if world > 1 else None,
            "synced": synced,
            "upload_s": upload_s,
            "loglik_last": st.last_log_likelihood,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(N, K, T, topo, args.cpu_seconds, seed, args.symbols, args.cpu_threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def synced_protocol(eng, stats, world, dist, R, iters=10, dropin_iters=20):
    """median of `iters` EM iterations, each followed by the host's read-back of the
    convergence record (hmm_training.py:503-514), plus the drop-in train loop (BaumWelchEngine.train:
    chunked status syncs) over `dropin_iters` iterations, in ms per iteration.

    The M-step of iteration e runs in the prologue of launch e + 1, so the record the host reads after
    enqueueing launch e + 1 is iteration e's, and the host decides on it before enqueueing launch e + 2.
    live (the headline synced figure, HMMBW_OPT_LIVE_STATUS): that prologue also writes the record into
    pinned host memory, which the host polls (hmmbw_status_live_wait), so the read-back overlaps the rest of
    launch e + 1.  snapshot: after each launch hmmbw_status_post enqueues a status snapshot kernel and the
    host waits for that snapshot (the launch's end) before enqueueing again.
    flush (kept for comparison): hmmbw_get_status after each iteration, which first runs the pending
    M-step as its own kernel and synchronises the stream."""
    import torch
    eng.status()
    base = eng.status()[0].iterations
    # live (the headline): the M-step in launch e + 1's prologue writes iteration e's record into pinned
    # host memory while that launch runs; the host polls it (hmmbw_status_live_wait) and enqueues the
    # next launch as soon as it has read it, so the record of every iteration is read back before the
    # iteration after next starts and the GPU never waits for the host
    eng.live_status(True)
    per_live = []
    for k in range(iters + 1):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        eng.enqueue_iterations(1, stats)
        if k >= 1:
            st, _ = eng.wait_live(base + k)  # iteration base + k - 1's record, from this launch's prologue
            per_live.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    eng.live_status(False)
    base = eng.status()[0].iterations
    per = []
    for k in range(iters):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        eng.enqueue_iterations(1, stats)
        first = max(base + k - 1, 0)  # the record of the iteration whose M-step this launch ran
        tk = eng.post_status(first)
        st, _ = eng.wait_status(tk, first)  # the snapshot's pinned record, no stream-wide sync
        per.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    per_flush = []
    for _ in range(iters):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        eng.enqueue_iterations(1, stats)
        eng.status()  # the pending M-step as its own kernel, then the D2H (synchronises the engine stream)
        per_flush.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    st = eng.train(0.0, dropin_iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    med = float(np.median(per))
    med_live = float(np.median(per_live))
    if world > 1:
        t = torch.tensor([med, dt, med_live], dtype=torch.float64,
                         device=f"cuda:{eng.device}" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        med, dt, med_live = float(t[0]), float(t[1]), float(t[2])
    return {"median_ms_per_iter_with_d2h": 1000.0 * med_live, "utt_per_s_with_d2h": R * world / med_live,
            "protocol": "live: per iteration one launch, then the host polls the pinned convergence record that "
                        "the next launch's merged M-step writes (hmmbw_status_live_wait) before enqueueing again",
            "median_ms_per_iter_snapshot": 1000.0 * med,
            "protocol_snapshot": "launch + status snapshot kernel (hmmbw_status_post/_wait) per iteration",
            "median_ms_per_iter_with_flush": 1000.0 * float(np.median(per_flush)),
            "dropin_train_ms_per_iter": 1000.0 * dt / max(st.iterations, 1), "dropin_iterations": st.iterations}


def dry_run(args, world, rank, wl, R, T, N, K, topo):
    """No GPU: the process group, barrier and max-over-ranks timing of the real run around a no-op."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo" if args.dist_backend == "gloo" else args.dist_backend)
        dist.barrier()
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": f"Baum-Welch utterances/sec/iter (T={T},N={N},K={K})", "value": None,
                          "unit": "utterances/s/iter", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "f64", "data": "dry run (no GPU work)",
                          "config": {"workload": wl, "sequences_per_gpu": R, "sequences_total": R * world, "T": T,
                                     "N": N, "K": K, "topology": topo,
                                     "parallelism": f"dp{world}" if world > 1 else "single"},
                          "roofline": None, "cpu_baseline": None, "dry_run_barrier_s": elapsed}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
