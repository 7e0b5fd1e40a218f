"""Round 6 diagnostic: where do the peer all-reduce's sums go wrong for the wide path with uncached regions?

Runs the in-process peer cases of tests/test_gpu_peer.py in the suite's order (each memory kind in turn, as
the parametrisation orders them) up to the failing case, then that case with every buffer captured:
  X_r     rank r's pushed payload (hmmbw_iterate_begin's buffer), copied right after its E-step
  slot_qr rank r's receive region, slot q of the iteration's parity, after all pushes / after all reduces
and compares slot_qr with X_q (did the push land?) and the M-step's parameters with the fixture.
Prints one JSON line per checked iteration.

    python tools/peer_diag.py [--until n64_k1024_tiny] [--world 2] [--kinds coarse,uncached] [--skip-history]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--until", default="n64_k1024_tiny")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--kinds", default="coarse,uncached")
    ap.add_argument("--skip-history", action="store_true")
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    import test_gpu_peer as T
    from hmm_training_amd.engine import BaumWelchEngine, shard_bounds
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipDeviceSynchronize.argtypes = []

    def d2h(ptr, n):
        out = np.empty(n, dtype=np.float64)
        hip.hipDeviceSynchronize()
        assert hip.hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), 8 * n, 2) == 0
        return out

    kinds = a.kinds.split(",")
    if not a.skip_history:  # the suite's order: case, world, deterministic, kind
        for case in T.CASES:
            if case == a.until:
                break
            for world in (2, 3, 8):
                for det in (False, True):
                    for kind in kinds:
                        os.environ["HMMBW_PEER_MEM"] = kind
                        d = T.load(case)
                        bounds, out = T.run_world_peer(d, world, det)
                        ok = all(np.all(np.abs(o[3][1] - d["out_A"]) <= 1e-6 * np.abs(d["out_A"]) + 1e-15) for o in out)
                        print(json.dumps({"history": case, "world": world, "det": det, "kind": kind, "A_ok": bool(ok)}),
                              flush=True)
    d = T.load(a.until)
    N, M = int(d["N"]), int(d["M"])
    obs = T.observations(d)
    for kind in kinds:
        os.environ["HMMBW_PEER_MEM"] = kind
        bounds = shard_bounds([len(o) for o in obs], a.world)
        engines = []
        try:
            for r, (lo, hi) in enumerate(bounds):
                e = BaumWelchEngine(N, M, rank=r, world_size=a.world)
                e.set_observations(obs[lo:hi], n_seq_global=len(obs))
                e.set_params(d["init_pi"], d["init_A"], d["init_B"])
                e.reset(float(d["epsilon"]), int(d["max_iterations"]))
                engines.append(e)
            T.attach_in_process(engines)
            regions = []
            for e in engines:
                ptr, nb = ctypes.c_void_p(), ctypes.c_int64()
                e._lib.hmmbw_peer_region(e._ctx, ctypes.byref(ptr), ctypes.byref(nb))
                regions.append((ptr.value, nb.value))
            for it in range(int(d["max_iterations"]) + 1):
                bufs = []
                for e in engines:
                    ptr, n = e.iterate_begin()
                    bufs.append((ptr, n))
                X = [d2h(p, n) for p, n in bufs]
                n = bufs[0][1]
                slot = (n + 31) // 32 * 32
                par = (it + 1) & 1  # peer_seq starts at 1
                rep = {"kind": kind, "iteration": it, "n": n, "regions": [hex(p) for p, _ in regions],
                       "bufs": [hex(p) for p, _ in bufs]}
                nd = regions[0][1] // 8
                pushed = []
                for r, (rp, nb) in enumerate(regions):
                    reg = d2h(rp, nb // 8)
                    for q in range(a.world):
                        s = reg[(par * a.world + q) * slot:(par * a.world + q) * slot + n]
                        bad = np.flatnonzero(s != X[q])
                        pushed.append({"region": r, "slot": q, "n_bad": int(bad.size),
                                       "first_bad": int(bad[0]) if bad.size else None,
                                       "sum_X": float(X[q].sum()), "sum_slot": float(s.sum())})
                rep["after_push"] = pushed
                for e in engines:
                    e.iterate_end()
                hip.hipDeviceSynchronize()
                ref_sum = X[0].copy()
                for q in range(1, a.world):
                    ref_sum = ref_sum + X[q]
                xs = []
                for r, e in enumerate(engines):
                    xp = e.get_option(110)
                    got = d2h(xp, n)
                    bad = np.flatnonzero(got != ref_sum)
                    xs.append({"rank": r, "xsum": hex(xp), "n_bad": int(bad.size), "first_bad": bad[:8].tolist(),
                               "got": got[bad[:4]].tolist(), "want": ref_sum[bad[:4]].tolist()})
                rep["xsum"] = xs
                after = []
                for r, (rp, nb) in enumerate(regions):
                    reg = d2h(rp, nb // 8)
                    for q in range(a.world):
                        s = reg[(par * a.world + q) * slot:(par * a.world + q) * slot + n]
                        bad = np.flatnonzero(s != X[q])
                        after.append({"region": r, "slot": q, "n_bad": int(bad.size),
                                      "first_bad": int(bad[0]) if bad.size else None})
                    fl = reg[2 * a.world * slot:].view(np.uint64)
                    after.append({"region": r, "flags": [int(x) for x in fl[:64]]})
                rep["after_reduce"] = after
                print(json.dumps(rep), flush=True)
            for r, e in enumerate(engines):
                pi, A, B = e.params(normalise=True)
                err = np.abs(A - d["out_A"]) - (1e-6 * np.abs(d["out_A"]) + 1e-15)
                errB = np.abs(B - d["out_B"]) - (1e-6 * np.abs(d["out_B"]) + 1e-15)
                rows = sorted(set(int(i) for i in np.argwhere(err > 0)[:, 0]))
                print(json.dumps({"kind": kind, "rank": r, "A_worst": float(err.max()), "B_worst": float(errB.max()),
                                  "bad_A_rows": rows[:64]}), flush=True)
        finally:
            for e in engines:
                e.close()


if __name__ == "__main__":
    main()
