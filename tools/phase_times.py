#!/usr/bin/env python3
"""Per-wave phase timeline of the small E-step (diagnostics).

Builds an instrumented copy of the engine (-DHMMBW_PHASE_TIMES) into gpurun_out/, runs the bench
workload for a few iterations and prints, for the last launch, the distribution over waves of each
phase's duration and of the phase boundaries relative to the earliest wave start (wall clock, 100 MHz).

    python tools/phase_times.py [--R 10000] [--topology left_to_right] [--no-merge]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", default="10000", help="comma-separated sequence counts")
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--N", type=int, default=8)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--topology", default="left_to_right")
    ap.add_argument("--no-merge", action="store_true")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--prewarm", type=int, default=3000, help="untimed iterations first (GPU clock ramp)")
    ap.add_argument("--kwaves", type=int, default=0, help="kernel waves to read (default: R / sequences per wave)")
    ap.add_argument("--lib", default=None, help="prebuilt diagnostics library (default hmm_training_amd/libhmmbw_phase.so)")
    ap.add_argument("--json", default=None, help="write the per-class phase summary (busy / lone SIMDs) here")
    ap.add_argument("--chunks", action="store_true", help="also stamp every chunk (-DHMMBW_CHUNK_TIMES; per-class chunk cycles)")
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out", "phase")
    os.makedirs(out_dir, exist_ok=True)
    name = "libhmmbw_chunk.so" if a.chunks else "libhmmbw_phase.so"
    lib = a.lib or os.path.join(ROOT, "hmm_training_amd", name)  # prebuilt in-tree if present
    if not os.path.exists(lib):
        from hmm_training_amd import build as B
        defs = ["-DHMMBW_PHASE_TIMES"] + (["-DHMMBW_CHUNK_TIMES"] if a.chunks else [])
        B.build(force=True, defines=defs, out=lib, tag="chunk" if a.chunks else "phase")
    os.environ["HMMBW_LIB"] = lib
    import torch
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    for R in [int(x) for x in a.R.split(",")]:
        run_one(a, R, torch, BaumWelchEngine, default_initial_params, out_dir)


def run_one(a, R, torch, BaumWelchEngine, default_initial_params, out_dir):
    print(f"==== R={R}")
    T, N, K = a.T, a.N, a.K
    rng = np.random.default_rng(3)
    sym = rng.integers(0, K, size=R * T).astype(np.int32)
    pi, A, Bm = default_initial_params(N, K)
    if a.topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    eng = BaumWelchEngine(N, K, topology=a.topology, merge_mstep=not a.no_merge)
    eng.set_observations(offsets=np.arange(R + 1, dtype=np.int64) * T, symbols=sym)
    eng.set_params(pi, A, Bm)
    if a.prewarm > 0:
        eng.reset(0.0, a.prewarm + 1)
        eng.enqueue_iterations(a.prewarm)
        torch.cuda.synchronize()
    eng.reset(0.0, a.iters + 1)
    eng.enqueue_iterations(a.iters)
    torch.cuda.synchronize()
    U = 64 // (1 << max(1, (N - 1).bit_length()))
    nw = (R + U - 1) // U
    if a.kwaves:
        nw = a.kwaves
    nw_pad = ((nw + 3) // 4) * 4
    buf = np.zeros((nw_pad, 16), dtype=np.uint64)
    l = eng._lib
    l.hmmbw_debug_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    rc = l.hmmbw_debug_phase_times(buf.ctypes.data, nw_pad)
    assert rc == 0, rc
    t = buf[:nw].astype(np.int64)
    t0 = t[:, 0].min()
    us = lambda x: x / 100.0  # 100 MHz wall clock -> us
    names = ["start", "tables", "forward", "backward", "ll", "flush"]
    print(f"waves {nw}  kernel span {us(t[:, 5].max() - t0):.2f} us")
    # waves that never stamp a phase in this launch (the idle waves of the spread map's xact-wave
    # workgroups: their slots hold an earlier launch's stamps) are left out of that phase's statistics
    for k in range(1, 6):
        ok = (t[:, k] >= t0) & (t[:, k - 1] >= t0)
        d = us(t[ok, k] - t[ok, k - 1])
        print(f"{names[k-1]:>8s}->{names[k]:<8s} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")
    for k in range(6):
        r = us(t[t[:, k] >= t0, k] - t0)
        print(f"at {names[k]:<8s} rel-start  min {r.min():7.2f}  p50 {np.median(r):7.2f}  max {r.max():7.2f} us")
    if np.all(t[:, 6] > 0):  # merged M-step prologue: statistics gathered / tables built
        for k, nm in ((13, "zero-cleared"), (8, "mstep-entry"), (9, "stats-landed"), (6, "mstep-loads"),
                      (7, "mstep-sum"), (10, "tables-written"), (11, "hist-flushed")):
            r = us(t[:, k] - t0)
            print(f"at {nm:<12s} rel-start  min {r.min():7.2f}  p50 {np.median(r):7.2f}  max {r.max():7.2f} us")
    np.save(os.path.join(out_dir, "phase_nomerge.npy" if a.no_merge else "phase_merge.npy"), t)
    if a.json:
        write_json(a, R, eng, l, us)
    # per-chunk shader-clock durations (forward: chunk c -> c+1; backward: chunk c -> c-1)
    ck = np.zeros((nw_pad, 2, 64), dtype=np.uint64)
    l.hmmbw_debug_chunk_times.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert l.hmmbw_debug_chunk_times(ck.ctypes.data, nw_pad) == 0
    ck = ck[:nw].astype(np.int64)
    if not np.any(ck):
        return  # chunk stamps need -DHMMBW_CHUNK_TIMES as well
    nch = (T + 7) // 8
    fwd = np.diff(ck[:, 0, :nch], axis=1)
    bwd = -np.diff(ck[:, 1, :nch], axis=1)  # stamped in descending chunk order
    span_clk = (ck[:, 0, nch - 1] - ck[:, 0, 0]).astype(float)
    span_us = us((t[:, 2] - t[:, 1]).astype(float))
    print(f"forward chunk cycles: p50 {np.median(fwd):.0f}  mean {fwd.mean():.0f}  max {fwd.max():.0f}; per chunk p50 over waves: "
          + " ".join(f"{np.median(fwd[:, c]):.0f}" for c in range(min(fwd.shape[1], 12))))
    print(f"backward chunk cycles: p50 {np.median(bwd):.0f}  mean {bwd.mean():.0f}  max {bwd.max():.0f}")
    print(f"shader clock estimate: {np.median(span_clk / np.maximum(span_us * (nch - 1) / nch, 1e-9)) / 1e3:.2f} GHz")


def write_json(a, R, eng, l, us):
    """Phase durations by SIMD class on the engine's launch map (bench.py's phase model reads this): `busy` =
    the waves on SIMDs that hold two sequence-group waves (joined map: full waves 0 .. xact-1 and extra waves
    4 .. 3+xact of the workgroups that carry extra groups; with split extra groups every full wave of those
    workgroups, their A and B waves in classes of their own), `lone` = the other full waves.  Stamps are indexed
    by (workgroup, wave) of the launched kernel: 8 waves per workgroup on the joined map."""
    import json
    import time
    sys.path.insert(0, ROOT)
    import bench
    m = eng.launch_map()
    joined = bool(m.get("joined"))
    wpw = 8 if joined else m["waves_per_workgroup"]
    nwg = m["full_workgroups"] if joined else m["workgroups"]
    xact = m["extra_waves"] or 4
    nx_groups = m["waves"] - m["full_workgroups"] * 4
    nx_wg = -(-nx_groups // xact) if nx_groups > 0 else 0
    n = ((nwg * wpw + 3) // 4) * 4
    buf = np.zeros((n, 16), dtype=np.uint64)
    assert l.hmmbw_debug_phase_times(buf.ctypes.data, n) == 0
    t = buf[:nwg * wpw].astype(np.int64)
    t0 = t[t[:, 0] > 0, 0].min()
    split = joined and bool(m.get("split_extra"))
    busy, lone, split_a, split_b = [], [], [], []
    busy_a, busy_b = [], []  # split: the full waves that share a SIMD with an A wave / with a B wave (waves w, w + 4)
    for b in range(nwg):
        for wv in range(wpw):
            idx = b * wpw + wv
            if joined and split and b < nx_wg:
                # split extra groups: A waves 4 .. 3+xact (SIMDs 0 ..), B waves 4+xact .. 3+2 xact; every full
                # wave of the workgroup shares its SIMD with one of them
                if wv < 4:
                    busy.append(idx)
                    if wv < xact:
                        busy_a.append(idx)
                    elif wv < 2 * xact:
                        busy_b.append(idx)
                elif wv < 4 + xact:
                    split_a.append(idx)
                elif wv < 4 + 2 * xact:
                    split_b.append(idx)
            elif joined:
                if b < nx_wg and (wv < xact or 4 <= wv < 4 + xact):
                    busy.append(idx)
                elif wv < 4:
                    lone.append(idx)
            elif wv < 4:
                lone.append(idx)
    out = {"tool": "tools/phase_times.py --json", "R": R, "T": a.T, "N": a.N, "K": a.K, "topology": a.topology,
           "launch_map": m, "kernel_src_sha16": bench.kernel_source_hash(),
           "collected_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "span_us": float(us(t[:, 5].max() - t0)), "classes": {}}
    names = ["start", "tables", "forward", "backward", "ll", "flush"]
    for cls, ids in (("busy", busy), ("lone", lone), ("split_a", split_a), ("split_b", split_b),
                     ("busy_with_a", busy_a), ("busy_with_b", busy_b)):
        if not ids:
            continue
        tt = t[ids]
        tt = tt[(tt[:, 0] >= t0) & (tt[:, 5] >= t0)]
        c = {"waves": int(len(tt))}
        for k in range(1, 6):
            d = us(tt[:, k] - tt[:, k - 1])
            c[f"{names[k-1]}->{names[k]}_us"] = {"p50": float(np.median(d)), "max": float(d.max())}
        for k in range(6):
            r = us(tt[:, k] - t0)
            c[f"at_{names[k]}_us"] = {"p50": float(np.median(r)), "max": float(r.max())}
        out["classes"][cls] = c
    # per-class chunk cycles (chunk-stamp build): forward chunk c -> c+1, backward chunk c -> c-1 (descending)
    nck = n if n <= 4096 else 4096
    ck = np.zeros((4096, 2, 64), dtype=np.uint64)
    if hasattr(l, "hmmbw_debug_chunk_times"):
        l.hmmbw_debug_chunk_times.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        if l.hmmbw_debug_chunk_times(ck.ctypes.data, 4096) == 0 and np.any(ck):
            ck = ck.astype(np.int64)
            nch = (a.T + 7) // 8
            out["chunk_cycles"] = {}
            for cls, ids in (("busy", busy), ("lone", lone), ("split_a", split_a), ("split_b", split_b)):
                ids = [i for i in ids if i < nck and np.all(ck[i, 0, :nch] > 0)]
                if not ids:
                    continue
                f = np.diff(ck[ids, 0, :nch], axis=1)
                b = ck[ids, 1, :nch]
                db = b[:, :-1] - b[:, 1:]  # chunk c's stamp is later than chunk c + 1's
                ok = (b[:, :-1] > 0) & (b[:, 1:] > 0)
                out["chunk_cycles"][cls] = {
                    "waves": len(ids),
                    "forward_p50_per_chunk": [float(np.median(f[:, c])) for c in range(f.shape[1])],
                    "backward_p50_per_chunk": [float(np.median(db[ok[:, c], c])) if ok[:, c].any() else None
                                               for c in range(db.shape[1])]}
    # where the waves ran (slot 15 = HW_ID: SIMD bits 5:4, CU bits 11:8, shader array 12, engine 15:13; slot 14 = XCC)
    hw = t[:, 15]
    if np.any(hw):
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        maps = {}
        for b in range(min(nwg, 512)):
            key = tuple(int(x) for x in simd[b * wpw:(b + 1) * wpw])
            maps[key] = maps.get(key, 0) + 1
        out["wave_simd_maps"] = [{"simd_of_wave": list(k), "workgroups": v} for k, v in sorted(maps.items(), key=lambda kv: -kv[1])]
        same_cu = sum(1 for b in range(nwg) if len(set(int(x) for x in cu[b * wpw:(b + 1) * wpw])) == 1)
        out["workgroups_on_one_cu"] = same_cu
        print("wave -> SIMD maps of the workgroups (count):", out["wave_simd_maps"][:4])
    with open(a.json, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", a.json)


if __name__ == "__main__":
    main()
