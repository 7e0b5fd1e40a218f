"""ctypes wrapper over oracle/liboracle.so (bw_oracle.c).  TEST INFRASTRUCTURE ONLY.

The parity checker for the MI355X Baum-Welch build: a fp64 log-domain CPU restatement of
DemianMArin/HMM_Training HMM/hmm_training.py:265-541 and hmm_testing.py:49-104.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The product
package (hmm_training_amd/) never does.

Build with ``python oracle/build_oracle.py`` (also run by ``__graft_entry__.build()``).
Pinned against tests/golden/*.npz (generated from the reference) by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            from oracle.build_oracle import build
            build()
        lib = ctypes.CDLL(LIB_PATH)
        lib.oracle_hmm_training.restype = ctypes.c_int64
        lib.oracle_hmm_training.argtypes = [_ip, _ip, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                            ctypes.c_int64, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                                            _dp]
        lib.oracle_estep_logstats.restype = ctypes.c_int
        lib.oracle_estep_logstats.argtypes = [_ip, _ip, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp,
                                              _dp, _dp, _dp, _dp, _dp, _dp]
        lib.oracle_forward_loglik.restype = ctypes.c_int
        lib.oracle_forward_loglik.argtypes = [_ip, _ip, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp,
                                              _dp]
        lib.oracle_vq.restype = None
        lib.oracle_vq.argtypes = [_dp, ctypes.c_int64, _dp, ctypes.c_int64, ctypes.c_int, _ip, _dp]
        lib.oracle_lse.restype = ctypes.c_double
        lib.oracle_lse.argtypes = [_dp, ctypes.c_int64]
        lib.oracle_set_threads.restype = ctypes.c_int
        lib.oracle_set_threads.argtypes = [ctypes.c_int]
        lib.oracle_mstep_log.restype = None
        lib.oracle_mstep_log.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp,
                                         _dp, _dp]
        _lib = lib
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the E-step (over utterances); 1 = the serial restatement the parity tests
    use.  Returns the count in effect.  Only bench.py's cpu_baseline leg raises it."""
    return int(load().oracle_set_threads(int(n)))


def to_csr(observations: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    lengths = np.array([len(o) for o in observations], dtype=np.int64)
    offsets = np.zeros(len(observations) + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    symbols = (np.concatenate([np.asarray(o, dtype=np.int64) for o in observations])
               if len(observations) else np.zeros(0, np.int64))
    return offsets, np.ascontiguousarray(symbols, dtype=np.int64)


def safe_log(x):
    x = np.asarray(x, dtype=np.float64)
    out = np.full_like(x, -np.inf)
    m = x > 0
    out[m] = np.log(x[m])
    return out


class OracleResult:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def hmm_training(offsets, symbols, N, M, epsilon, max_iterations, pi0, A0, B0) -> OracleResult:
    """Run the oracle's restatement of hmm_training.py:265-541 from linear initial params."""
    lib = load()
    R = len(offsets) - 1
    out_A = np.zeros((N, N)); out_B = np.zeros((N, M)); out_pi = np.zeros(N)
    nt = max(int(max_iterations), 1)
    tL = np.zeros(nt); tD = np.zeros(nt)
    logP = np.zeros(max(R, 1)); lpi = np.zeros(N); la = np.zeros((N, N)); lb = np.zeros((N, M))
    it = lib.oracle_hmm_training(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(symbols, np.int64),
                                 R, N, M, float(epsilon), int(max_iterations),
                                 np.ascontiguousarray(pi0, np.float64), np.ascontiguousarray(A0, np.float64),
                                 np.ascontiguousarray(B0, np.float64), out_A, out_B, out_pi, tL, tD, logP, lpi,
                                 la, lb)
    if it < 0:
        raise RuntimeError(f"oracle_hmm_training failed ({it})")
    return OracleResult(A=out_A, B=out_B, pi=out_pi, iterations=int(it), trace_L=tL[:it], trace_diff=tD[:it],
                        logP=logP[:R], log_pi=lpi, log_A=la, log_B=lb)


def estep_logstats(offsets, symbols, N, M, pi, A, B) -> OracleResult:
    """Log-domain E-step sufficient statistics for LINEAR params (pi, A, B)."""
    lib = load()
    R = len(offsets) - 1
    lpi_num = np.zeros(N); lxi = np.zeros((N, N)); lgex = np.zeros(N); lgall = np.zeros(N)
    lbnum = np.zeros((N, M)); logP = np.zeros(max(R, 1))
    rc = lib.oracle_estep_logstats(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(symbols, np.int64),
                                   R, N, M, safe_log(pi), safe_log(A), safe_log(B), lpi_num, lxi, lgex, lgall,
                                   lbnum, logP)
    if rc != 0:
        raise RuntimeError(f"oracle_estep_logstats failed ({rc})")
    return OracleResult(log_pi_num=lpi_num, log_xi=lxi, log_gden_excl=lgex, log_gden_all=lgall, log_bnum=lbnum,
                        logP=logP[:R])


def merge_logstats(parts) -> OracleResult:
    """E-step statistics of a set of sequences from those of a partition of it (each an estep_logstats
    result): every statistic is a log-sum over sequences (hmm_training.py:415-497), so the parts combine by
    log-sum-exp (-inf parts drop out, as in the reference's log_sum_exp, :66-79); logP concatenated."""
    def lse_all(name):
        with np.errstate(invalid="ignore"):
            return np.logaddexp.reduce(np.stack([getattr(p, name) for p in parts]), axis=0)
    return OracleResult(log_pi_num=lse_all("log_pi_num"), log_xi=lse_all("log_xi"),
                        log_gden_excl=lse_all("log_gden_excl"), log_gden_all=lse_all("log_gden_all"),
                        log_bnum=lse_all("log_bnum"), logP=np.concatenate([p.logP for p in parts]))


def mstep_log(R, N, M, s: OracleResult):
    """The reference's M-step (hmm_training.py:415-500) from log statistics: (log_pi, log_A, log_B),
    unnormalised, R counting every sequence (:424)."""
    lpi, la, lb = np.zeros(N), np.zeros(N * N), np.zeros(N * M)
    load().oracle_mstep_log(int(R), N, M, np.ascontiguousarray(s.log_pi_num, np.float64),
                            np.ascontiguousarray(s.log_xi, np.float64).reshape(-1),
                            np.ascontiguousarray(s.log_gden_excl, np.float64),
                            np.ascontiguousarray(s.log_gden_all, np.float64),
                            np.ascontiguousarray(s.log_bnum, np.float64).reshape(-1), lpi, la, lb)
    return lpi, la.reshape(N, N), lb.reshape(N, M)


def forward_loglik(offsets, symbols, N, M, pi, A, B) -> np.ndarray:
    lib = load()
    R = len(offsets) - 1
    out = np.zeros(max(R, 1))
    rc = lib.oracle_forward_loglik(np.ascontiguousarray(offsets, np.int64), np.ascontiguousarray(symbols, np.int64),
                                   R, N, M, np.ascontiguousarray(pi, np.float64),
                                   np.ascontiguousarray(A, np.float64), np.ascontiguousarray(B, np.float64), out)
    if rc != 0:
        raise RuntimeError(f"oracle_forward_loglik failed ({rc})")
    return out[:R]


def vq(frames: np.ndarray, centroids: np.ndarray, return_dist: bool = False):
    """Nearest-centroid index over columns [1, D) (hmm_training.py:82-120); frames [F][D], centroids [K][D]."""
    lib = load()
    frames = np.ascontiguousarray(frames, np.float64)
    centroids = np.ascontiguousarray(centroids, np.float64)
    out = np.zeros(len(frames), dtype=np.int64)
    dist = np.zeros(len(frames), dtype=np.float64)
    lib.oracle_vq(frames, len(frames), centroids, len(centroids), frames.shape[1], out, dist)
    return (out, dist) if return_dist else out


def lse(x) -> float:
    x = np.ascontiguousarray(x, np.float64)
    return float(load().oracle_lse(x, len(x)))
