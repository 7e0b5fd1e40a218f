"""ctypes binding of libhmmbw.so (include/hmmbw.h).

The HIP engine is the only compute path: if the shared library is missing or fails to load, every
entry point raises (there is no CPU fallback).  torch is imported first so that the HIP runtime
(libamdhip64.so.7) loaded by torch is the one the engine binds to — one runtime per process, so
torch streams/tensors and the engine's kernels interoperate.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HMMBW_LIB", os.path.join(PKG_DIR, "libhmmbw.so"))

HMMBW_OK = 0
HMMBW_E_INVALID = -1
HMMBW_E_HIP = -2
HMMBW_E_UNSUPPORTED = -3
HMMBW_E_STATE = -4
HMMBW_E_EMPTY_SEQUENCE = -5
HMMBW_E_SYMBOL_RANGE = -6
HMMBW_E_TIMEOUT = -7

TOPOLOGY = {"auto": 0, "dense": 1, "left_to_right": 2}
TOPOLOGY_NAME = {v: k for k, v in TOPOLOGY.items()}

# every symbol include/hmmbw.h declares (tests check the library exports all of them)
EXPORTED = (
    "hmmbw_abi_version", "hmmbw_last_error", "hmmbw_device_count", "hmmbw_ctx_create", "hmmbw_ctx_destroy",
    "hmmbw_set_stream", "hmmbw_set_rank", "hmmbw_set_topology", "hmmbw_get_topology", "hmmbw_set_observations",
    "hmmbw_set_params", "hmmbw_reset_training", "hmmbw_stats_len", "hmmbw_estep", "hmmbw_mstep",
    "hmmbw_iterate", "hmmbw_get_status", "hmmbw_status_post", "hmmbw_status_wait",
    "hmmbw_get_params", "hmmbw_get_loglik", "hmmbw_score", "hmmbw_timing",
    "hmmbw_set_option", "hmmbw_group_create", "hmmbw_group_destroy", "hmmbw_group_iterate", "hmmbw_group_score",
    "hmmbw_group_timing", "hmmbw_vq_encode", "hmmbw_comm_unique_id", "hmmbw_comm_init",
    "hmmbw_comm_probe", "hmmbw_comm_info", "hmmbw_comm_payload", "hmmbw_iterate_begin", "hmmbw_iterate_end",
    "hmmbw_cache_trim", "hmmbw_timing_split", "hmmbw_peer_region", "hmmbw_peer_ipc_handle", "hmmbw_peer_open",
    "hmmbw_peer_attach", "hmmbw_allreduce_kind", "hmmbw_status_live_wait", "hmmbw_get_option",
)
ABI_VERSION = 5
OPT_SAFE_SCALING = 1
OPT_ABLATE = 2
OPT_STAT_COPIES = 3
OPT_MERGE_MSTEP = 4
OPT_DETERMINISTIC = 7
OPT_ALLREDUCE = 8
OPT_PEER_TIMEOUT_MS = 9
OPT_LIVE_STATUS = 10
OPT_WQ_TIMEOUT_MS = 11
OPT_WIDE_WQ = 12
INFO_WIDE_WQ_ACTIVE = 101
INFO_WAVES = 102
INFO_WORKGROUPS = 103
INFO_WAVES_PER_WORKGROUP = 104
INFO_FULL_WORKGROUPS = 105
INFO_EXTRA_WAVES = 106
INFO_PEER_CHUNKS = 107
INFO_JOINED = 108
INFO_SPLIT_EXTRA = 109
ALLREDUCE = {"rccl": 0, "peer": 1}


class HMMBWError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hmmbw error {code}: {msg}")
        self.code = code


class IterRecord(ctypes.Structure):
    _fields_ = [("log_likelihood", ctypes.c_double), ("diff", ctypes.c_double)]


class Status(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int64), ("done", ctypes.c_int32), ("converged", ctypes.c_int32),
                ("last_log_likelihood", ctypes.c_double), ("last_diff", ctypes.c_double)]


_lock = threading.Lock()
_lib = None


def _declare(lib):
    c_ctx = ctypes.c_void_p
    P = ctypes.POINTER
    sig = {
        "hmmbw_abi_version": (ctypes.c_int, []),
        "hmmbw_last_error": (ctypes.c_char_p, []),
        "hmmbw_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "hmmbw_cache_trim": (ctypes.c_int, [P(ctypes.c_int64)]),
        "hmmbw_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, P(c_ctx)]),
        "hmmbw_ctx_destroy": (ctypes.c_int, [c_ctx]),
        "hmmbw_set_stream": (ctypes.c_int, [c_ctx, ctypes.c_void_p]),
        "hmmbw_set_rank": (ctypes.c_int, [c_ctx, ctypes.c_int, ctypes.c_int]),
        "hmmbw_set_topology": (ctypes.c_int, [c_ctx, ctypes.c_int]),
        "hmmbw_get_topology": (ctypes.c_int, [c_ctx, P(ctypes.c_int)]),
        "hmmbw_set_observations": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
        "hmmbw_set_params": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
        "hmmbw_reset_training": (ctypes.c_int, [c_ctx, ctypes.c_double, ctypes.c_int64]),
        "hmmbw_stats_len": (ctypes.c_int, [c_ctx, P(ctypes.c_int64)]),
        "hmmbw_estep": (ctypes.c_int, [c_ctx, ctypes.c_void_p]),
        "hmmbw_mstep": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_int64]),
        "hmmbw_iterate": (ctypes.c_int, [c_ctx, ctypes.c_int64]),
        "hmmbw_iterate_begin": (ctypes.c_int, [c_ctx, ctypes.c_int64, P(ctypes.c_void_p), P(ctypes.c_int64)]),
        "hmmbw_iterate_end": (ctypes.c_int, [c_ctx]),
        "hmmbw_get_status": (ctypes.c_int, [c_ctx, P(Status), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]),
        "hmmbw_status_post": (ctypes.c_int, [c_ctx, ctypes.c_int64, P(ctypes.c_int64)]),
        "hmmbw_status_wait": (ctypes.c_int, [c_ctx, ctypes.c_int64, P(Status), ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int64]),
        "hmmbw_status_live_wait": (ctypes.c_int, [c_ctx, ctypes.c_int64, P(Status), ctypes.c_void_p, ctypes.c_int64,
                                                  ctypes.c_int64]),
        "hmmbw_get_params": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
        "hmmbw_get_loglik": (ctypes.c_int, [c_ctx, ctypes.c_void_p]),
        "hmmbw_score": (ctypes.c_int, [c_ctx, ctypes.c_void_p]),
        "hmmbw_timing": (ctypes.c_int, [c_ctx, ctypes.c_int, P(ctypes.c_double), P(ctypes.c_int64)]),
        "hmmbw_timing_split": (ctypes.c_int, [c_ctx, P(ctypes.c_double), P(ctypes.c_int64)]),
        "hmmbw_peer_region": (ctypes.c_int, [c_ctx, P(ctypes.c_void_p), P(ctypes.c_int64)]),
        "hmmbw_peer_ipc_handle": (ctypes.c_int, [c_ctx, ctypes.c_void_p]),
        "hmmbw_peer_open": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_int64]),
        "hmmbw_peer_attach": (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_int64]),
        "hmmbw_allreduce_kind": (ctypes.c_int, [c_ctx, P(ctypes.c_int)]),
        "hmmbw_set_option": (ctypes.c_int, [c_ctx, ctypes.c_int, ctypes.c_int64]),
        "hmmbw_get_option": (ctypes.c_int, [c_ctx, ctypes.c_int, P(ctypes.c_int64)]),
        "hmmbw_vq_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]),
        "hmmbw_comm_probe": (ctypes.c_int, [ctypes.c_char_p]),
        "hmmbw_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p]),
        "hmmbw_comm_init": (ctypes.c_int, [c_ctx, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int64]),
        "hmmbw_comm_info": (ctypes.c_int, [c_ctx, P(ctypes.c_int), P(ctypes.c_double), P(ctypes.c_int64),
                                           ctypes.c_int]),
        "hmmbw_comm_payload": (ctypes.c_int, [c_ctx, P(ctypes.c_int64)]),
        "hmmbw_group_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_void_p)]),
        "hmmbw_group_destroy": (ctypes.c_int, [ctypes.c_void_p]),
        "hmmbw_group_iterate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
        "hmmbw_group_score": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
        "hmmbw_group_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_double), P(ctypes.c_int64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load libhmmbw.so (raises if it is missing: the HIP engine is mandatory)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libhmmbw.so not found at {LIB_PATH}: build it with `python -m hmm_training_amd.build` "
                    "(the MI355X engine has no CPU fallback)")
            handle = ctypes.CDLL(LIB_PATH)
            _declare(handle)
            v = handle.hmmbw_abi_version()
            if v != ABI_VERSION:
                raise ImportError(f"libhmmbw ABI version {v} != {ABI_VERSION} (stale build: rebuild with "
                                  "`python -m hmm_training_amd.build`)")
            _lib = handle
    return _lib


def cache_trim() -> int:
    """Return the library's cached device / pinned blocks to the driver (hmmbw_cache_trim); bytes freed."""
    n = ctypes.c_int64()
    check(lib().hmmbw_cache_trim(ctypes.byref(n)))
    return n.value


def check(rc: int) -> None:
    """Map an hmmbw status to the exception the reference would raise for the same input."""
    if rc == HMMBW_OK:
        return
    msg = lib().hmmbw_last_error().decode(errors="replace")
    if rc in (HMMBW_E_EMPTY_SEQUENCE, HMMBW_E_SYMBOL_RANGE):
        # reference: numpy IndexError at hmm_training.py:360/:376 (hmm_testing.py:75)
        raise IndexError(msg)
    if rc == HMMBW_E_INVALID:
        raise ValueError(msg)
    raise HMMBWError(rc, msg)
