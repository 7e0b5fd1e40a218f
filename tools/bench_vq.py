#!/usr/bin/env python3
"""HIP VQ encoder (hmmbw_vq_encode, get_observations hmm_training.py:82-120) throughput: frames/s over
F frames x K centroids x 12 dims already in HBM, kernel time from HIP events on the launch stream.
Work per frame: K x 12 x (sub + fma) fp64 = 36 K flops; priced against the 78.6 TFLOP/s fp64 vector
peak.   python tools/bench_vq.py [--frames 2000000] [--K 256] [--reps 20]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2_000_000)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from hmm_training_amd._lib import check, lib
    rng = np.random.default_rng(0)
    cents = rng.normal(size=(a.K, 13)) * 4.0
    frames = cents[rng.integers(0, a.K, size=a.frames)] + rng.normal(size=(a.frames, 13))
    tf = torch.from_numpy(frames).cuda()
    tc = torch.from_numpy(cents).cuda()
    ts = torch.empty(a.frames, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    L = lib()

    def go():
        check(L.hmmbw_vq_encode(ctypes.c_void_p(st.cuda_stream), ctypes.c_void_p(tf.data_ptr()), a.frames, 13, 1, 12,
                                ctypes.c_void_p(tc.data_ptr()), a.K, ctypes.c_void_p(ts.data_ptr()), None))
    for _ in range(3):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        go()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    flops = 36.0 * a.K * a.frames
    print(json.dumps({"kernel": "k_vq_encode<12>", "frames": a.frames, "K": a.K, "ms": ms,
                      "frames_per_s": a.frames / (ms / 1e3), "tflops": flops / (ms / 1e3) / 1e12,
                      "frac_fp64_vector_peak": flops / (ms / 1e3) / 1e12 / 78.6,
                      "hbm_gbs": (a.frames * (104 + 4)) / (ms / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
