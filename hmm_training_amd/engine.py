"""Device engine around libhmmbw: one context per (GPU, model shape), data-parallel over ranks.

Single rank: iterations are enqueued in chunks with ``hmmbw_iterate`` (E-step kernel + M-step kernel
per iteration, no host round trip); the host synchronises once per chunk to read the convergence
records.  Iterations enqueued after convergence are device-side no-ops, so the result is exactly
the reference's stop rule (hmm_training.py:346).

Multiple ranks (one process per GPU, torch.distributed over RCCL): every rank owns a contiguous,
length-balanced shard of the sequences; per iteration it runs the E-step on its shard, the packed
fp64 statistics are summed with ONE all-reduce, and every rank runs the identical M-step, so the
parameters and the convergence decision stay replicated without a broadcast.
With the nccl backend the engine gets its own RCCL communicator (hmmbw_comm_init) and the whole
estep -> all-reduce -> mstep sequence is enqueued by hmmbw_iterate on the engine's stream;
otherwise (gloo, or HMMBW_NATIVE_COMM=0) the all-reduce goes through torch.distributed.
"""
from __future__ import annotations

import collections
import ctypes
import json
import os
import time
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import (ALLREDUCE, INFO_WIDE_WQ_ACTIVE, OPT_ALLREDUCE, OPT_DETERMINISTIC, OPT_LIVE_STATUS, OPT_MERGE_MSTEP,
                   OPT_PEER_TIMEOUT_MS, OPT_SAFE_SCALING, OPT_STAT_COPIES, OPT_WIDE_WQ, OPT_WQ_TIMEOUT_MS, TOPOLOGY,
                   TOPOLOGY_NAME, IterRecord, Status, check, lib)

IterCallback = Callable[[int, float, float], None]


def to_csr(observations: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    """Ragged list of symbol arrays -> (offsets int64 [R+1], symbols int32 [sum T])."""
    arrs = [np.asarray(o).reshape(-1) for o in observations]
    lengths = np.fromiter((a.size for a in arrs), dtype=np.int64, count=len(arrs))
    offsets = np.zeros(len(arrs) + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    if len(arrs) and offsets[-1] > 0:
        sym = np.concatenate(arrs)
    else:
        sym = np.zeros(0, dtype=np.int64)
    if sym.size and not np.issubdtype(sym.dtype, np.integer):
        if not np.all(np.equal(np.mod(sym, 1), 0)):
            raise IndexError("observation symbols must be integers")
    return offsets, np.ascontiguousarray(sym, dtype=np.int32)


def shard_bounds(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous, length-balanced [start, end) shards of a sequence list (one per rank)."""
    lengths = np.asarray(lengths, dtype=np.int64)
    R = len(lengths)
    if world <= 1:
        return [(0, R)]
    cum = np.concatenate([[0], np.cumsum(lengths)])
    total = cum[-1]
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        idx = int(np.searchsorted(cum, target))
        if idx > 0 and abs(cum[idx - 1] - target) <= abs(cum[min(idx, R)] - target):
            idx -= 1
        idx = min(max(idx, cuts[-1]), R)
        cuts.append(idx)
    cuts.append(R)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


class StatsLayout:
    """Packed fp64 statistics buffer of hmmbw_estep/hmmbw_mstep (include/hmmbw.h):
    [pi_num N][xi N*N][gamma_den_excl_last N][gamma_den_all N][B_num M*N (symbol-major)][(m, s) x world].
    xi_ij = sum_r sum_t xi_t(i, j), the linear form of the reference's xi numerator
    (hmm_training.py:443-455); (m, s) is a rank's (max_r log P_r, sum_r exp(log P_r - m)) pair."""

    def __init__(self, N: int, M: int, world: int = 1):
        self.N, self.M, self.world = N, M, world
        self.pi = 0
        self.xi = N
        self.gex = N + N * N
        self.gall = self.gex + N
        self.bnum = self.gall + N
        self.ll = self.bnum + M * N
        self.length = self.ll + 2 * world

    def decode(self, buf: np.ndarray) -> dict:
        N, M = self.N, self.M
        buf = np.asarray(buf, dtype=np.float64)
        return dict(pi_num=buf[: N], xi=buf[self.xi: self.xi + N * N].reshape(N, N),
                    gamma_den_excl=buf[self.gex: self.gex + N], gamma_den_all=buf[self.gall: self.gall + N],
                    B_num=buf[self.bnum: self.bnum + M * N].reshape(M, N).T,
                    ll_pairs=buf[self.ll: self.ll + 2 * self.world].reshape(self.world, 2))

    @staticmethod
    def lse_of_pairs(pairs: np.ndarray) -> float:
        """L = LSE over all ranks' sequences from the per-rank (m, s) slots (mirrors k_mstep)."""
        pairs = np.asarray(pairs, dtype=np.float64).reshape(-1, 2)
        live = pairs[:, 1] > 0
        if not np.any(live):
            return float("-inf")
        m = np.max(pairs[live, 0])
        return float(m + np.log(np.sum(pairs[live, 1] * np.exp(pairs[live, 0] - m))))


def default_device() -> int:
    if torch.cuda.is_available():
        return torch.cuda.current_device()
    return 0


class BaumWelchEngine:
    """Baum-Welch training / scoring of one discrete HMM (N states, M symbols) on one GPU."""

    def __init__(self, n_states: int, n_symbols: int, device: Optional[int] = None, topology: str = "auto",
                 rank: int = 0, world_size: int = 1, stream: Optional[int] = None, safe_scaling: bool = False,
                 merge_mstep: bool = True, stat_copies: Optional[int] = None, group=None, native_comm: Optional[bool] = None,
                 deterministic: bool = False, allreduce: Optional[str] = None, peer_timeout_ms: Optional[int] = None):
        self._lib = lib()
        self.N, self.M = int(n_states), int(n_symbols)
        self.device = default_device() if device is None else int(device)
        self.rank, self.world_size = int(rank), int(world_size)
        ctx = ctypes.c_void_p()
        check(self._lib.hmmbw_ctx_create(self.device, self.N, self.M, ctypes.byref(ctx)))
        self._ctx = ctx
        if stream is None and torch.cuda.is_available():
            stream = torch.cuda.current_stream(self.device).cuda_stream
        if stream is not None:
            check(self._lib.hmmbw_set_stream(self._ctx, ctypes.c_void_p(stream)))
        if self.world_size > 1:
            check(self._lib.hmmbw_set_rank(self._ctx, self.rank, self.world_size))
        check(self._lib.hmmbw_set_topology(self._ctx, TOPOLOGY[topology]))
        if safe_scaling:
            check(self._lib.hmmbw_set_option(self._ctx, OPT_SAFE_SCALING, 1))
        if not merge_mstep:
            check(self._lib.hmmbw_set_option(self._ctx, OPT_MERGE_MSTEP, 0))
        if stat_copies is not None:  # None: the library default (2)
            check(self._lib.hmmbw_set_option(self._ctx, OPT_STAT_COPIES, int(stat_copies)))
        if deterministic:  # bitwise-reproducible statistics (no fp atomics); before set_observations
            check(self._lib.hmmbw_set_option(self._ctx, OPT_DETERMINISTIC, 1))
        self.n_seq = 0
        self.n_seq_global = 0
        self._group = group
        self._native = False   # multi-rank iterations through the engine's own RCCL communicator
        self._native_R = None
        if native_comm is None:
            native_comm = os.environ.get("HMMBW_NATIVE_COMM", "1") != "0"
        self._want_native = bool(native_comm) and self.world_size > 1
        # multi-rank all-reduce of the engine's own loop: "rccl" (engine communicator), "peer" (the engine's
        # push / wait + sum over IPC-mapped receive regions, hmmbw_peer_*), or "both" (set up both, RCCL
        # active; set_allreduce switches between iterations)
        self.allreduce_req = (allreduce or os.environ.get("HMMBW_ALLREDUCE", "rccl")).lower()
        if self.allreduce_req not in ("rccl", "peer", "both"):
            raise ValueError(f"allreduce must be rccl, peer or both, not {self.allreduce_req!r}")
        self._rccl_ok = False
        self._peer_ok = False
        if peer_timeout_ms is not None:
            check(self._lib.hmmbw_set_option(self._ctx, OPT_PEER_TIMEOUT_MS, int(peer_timeout_ms)))
        self._timing_mode = 0  # hmmbw_timing mode last set through timing()

    # -------------------------------------------------------------------------------- set-up
    def set_observations(self, observations: Sequence[np.ndarray] = None, offsets: np.ndarray = None,
                         symbols: np.ndarray = None, n_seq_global: Optional[int] = None) -> None:
        if observations is not None:
            offsets, symbols = to_csr(observations)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        symbols = np.ascontiguousarray(symbols, dtype=np.int32)
        R = len(offsets) - 1
        check(self._lib.hmmbw_set_observations(self._ctx, offsets.ctypes.data, symbols.ctypes.data, R))
        self.n_seq = R
        self.n_symbols_total = int(offsets[-1]) if R > 0 else 0
        self.n_seq_global = R if n_seq_global is None else int(n_seq_global)
        if self._want_native and self._native_R != self.n_seq_global:
            want_rccl = self.allreduce_req in ("rccl", "both")
            want_peer = self.allreduce_req in ("peer", "both")
            self._rccl_ok = self._init_native_comm() if want_rccl else False
            self._peer_ok = self._init_peer() if want_peer else False
            if self._rccl_ok and self.allreduce_req != "peer":
                self.set_allreduce("rccl")
            elif self._peer_ok:
                self.set_allreduce("peer")
            self._native = self._rccl_ok or self._peer_ok
            self._native_R = self.n_seq_global if self._native else None

    def set_allreduce(self, kind: str) -> None:
        """Switch the engine loop's all-reduce between iterations: "rccl" or "peer" (each must be set up)."""
        if kind == "rccl" and not self._rccl_ok:
            raise RuntimeError("the RCCL engine communicator is not set up")
        if kind == "peer" and not self._peer_ok:
            raise RuntimeError("the peer all-reduce is not set up")
        check(self._lib.hmmbw_set_option(self._ctx, OPT_ALLREDUCE, ALLREDUCE[kind]))

    @property
    def allreduce(self) -> Optional[str]:
        """The all-reduce the engine loop uses now: "rccl", "peer", or None (single rank / torch hop)."""
        k = ctypes.c_int()
        check(self._lib.hmmbw_allreduce_kind(self._ctx, ctypes.byref(k)))
        if k.value == ALLREDUCE["peer"]:
            return "peer"
        return "rccl" if (k.value == ALLREDUCE["rccl"] and self._native) else None

    def _agree(self, ok: bool) -> bool:
        """True iff every rank passes ok (an all-reduce MIN on the process group's device)."""
        import torch.distributed as dist
        dev = f"cuda:{self.device}" if dist.get_backend(self._group) == "nccl" else "cpu"
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self._group)
        return int(flag.item()) == 1

    def _init_peer(self) -> bool:
        """Collective over the ranks: the peer all-reduce (include/hmmbw.h, hmmbw_peer_*).  Every rank
        allocates its receive region, the 64-byte IPC handles are all-gathered over the process group (any
        backend), and every rank maps the others' regions; used only if every rank succeeded."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return False
        region, nbytes = ctypes.c_void_p(), ctypes.c_int64()
        handle = ctypes.create_string_buffer(64)
        ok = (self._lib.hmmbw_peer_region(self._ctx, ctypes.byref(region), ctypes.byref(nbytes)) == 0 and
              self._lib.hmmbw_peer_ipc_handle(self._ctx, handle) == 0)
        if not self._agree(ok):
            return False
        handles = [None] * dist.get_world_size(self._group)
        dist.all_gather_object(handles, handle.raw, group=self._group)
        buf = ctypes.create_string_buffer(b"".join(handles), 64 * len(handles))
        rc = self._lib.hmmbw_peer_open(self._ctx, buf, self.n_seq_global)
        # every rank must have attached (cleared its flags) before any rank pushes
        ok = self._agree(rc == 0)
        if ok:  # collective, so the count (the key of close()'s rendezvous) agrees across the ranks
            BaumWelchEngine._peer_setups += 1
            self._peer_tag = BaumWelchEngine._peer_setups
        return ok

    _peer_setups = 0  # peer set-ups of this process (every rank runs the same sequence)

    def _close_rendezvous(self, timeout_s: float) -> bool:
        """Bounded meeting of the ranks before the receive region is freed: each rank counts itself in under
        a key of the process group's store and waits (polling) until all have, or until timeout_s passes.
        Unlike dist.barrier, a rank that never arrives (it died, or closes at another point) cannot hold the
        others: they return False after the timeout and free their regions anyway (an IPC importer's mapping
        keeps the memory it writes alive until it closes the handle)."""
        import time
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
        key = f"hmmbw/peer_close/{self._peer_tag}"
        world = dist.get_world_size(self._group)
        store.add(key, 1)
        t_end = time.monotonic() + timeout_s
        delay = 1e-4
        while store.add(key, 0) < world:
            if time.monotonic() > t_end:
                return False
            time.sleep(delay)
            delay = min(2 * delay, 0.01)
        return True

    def _init_native_comm(self) -> bool:
        """Collective over the ranks: give the context its own RCCL communicator (hmmbw_comm_init), so
        multi-rank iterations run estep -> ncclAllReduce -> mstep on the engine's stream with no
        per-iteration host hop.  Every rank first checks it can resolve RCCL; unless all can, all
        keep the torch.distributed all-reduce path (no rank ever enters a collective alone)."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return False
        if dist.get_backend(self._group) != "nccl":
            return False
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        cpath = path.encode() if os.path.exists(path) else None
        uid = ctypes.create_string_buffer(128)
        ok = self._lib.hmmbw_comm_probe(cpath) == 0
        if ok and dist.get_rank(self._group) == 0:  # only the root creates the bootstrap id
            ok = self._lib.hmmbw_comm_unique_id(cpath, uid) == 0
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=f"cuda:{self.device}")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self._group)
        if int(flag.item()) == 0:
            return False
        obj = [uid.raw]
        src = dist.get_global_rank(self._group, 0) if self._group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=self._group, device=torch.device("cuda", self.device))
        rc = self._lib.hmmbw_comm_init(self._ctx, cpath, ctypes.c_char_p(obj[0]), self.rank, self.world_size,
                                       self.n_seq_global)
        # second agreement: the engine communicator is used only if every rank created it
        flag = torch.tensor([1 if rc == 0 else 0], dtype=torch.int32, device=f"cuda:{self.device}")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self._group)
        return int(flag.item()) == 1

    @property
    def native_comm(self) -> bool:
        return self._native

    def set_option(self, key: int, value: int) -> None:
        check(self._lib.hmmbw_set_option(self._ctx, int(key), int(value)))

    def get_option(self, key: int) -> int:
        v = ctypes.c_int64()
        check(self._lib.hmmbw_get_option(self._ctx, int(key), ctypes.byref(v)))
        return v.value

    def set_work_queue(self, mode: int, timeout_ms: Optional[int] = None) -> None:
        """Wide path (16 < N <= 64): HMMBW_OPT_WIDE_WQ (-1 auto from 4 tiles per CU, 0 off, 1 on when the
        tiles exceed the CUs) and the bound of its device-side wait (HMMBW_OPT_WQ_TIMEOUT_MS)."""
        self.set_option(OPT_WIDE_WQ, mode)
        if timeout_ms is not None:
            self.set_option(OPT_WQ_TIMEOUT_MS, timeout_ms)

    def launch_map(self) -> dict:
        """The E-step launch's wave map (HMMBW_INFO_*): active waves, workgroups, waves per workgroup, the
        workgroups with every wave active and the active waves of each workgroup after them; `joined`: the
        extra workgroups run as waves 4.. of the full ones (one 8-wave workgroup per CU); `split_extra`: the
        extra workgroups' idle waves run the lower backward half of their groups (dense)."""
        from ._lib import (INFO_EXTRA_WAVES, INFO_FULL_WORKGROUPS, INFO_JOINED, INFO_SPLIT_EXTRA, INFO_WAVES,
                           INFO_WAVES_PER_WORKGROUP, INFO_WORKGROUPS)
        return {"waves": self.get_option(INFO_WAVES), "workgroups": self.get_option(INFO_WORKGROUPS),
                "waves_per_workgroup": self.get_option(INFO_WAVES_PER_WORKGROUP),
                "full_workgroups": self.get_option(INFO_FULL_WORKGROUPS),
                "extra_waves": self.get_option(INFO_EXTRA_WAVES), "work_queue": self.work_queue_active,
                "joined": self.get_option(INFO_JOINED) == 1, "split_extra": self.get_option(INFO_SPLIT_EXTRA) == 1}

    def peer_chunks(self) -> int:
        """Chunks of the peer all-reduce payload (one flag per (rank, chunk) per iteration), 0 without a region."""
        from ._lib import INFO_PEER_CHUNKS
        return self.get_option(INFO_PEER_CHUNKS)

    @property
    def work_queue_active(self) -> bool:
        """True if the loaded observations' E-step runs on the wide work queue (HMMBW_INFO_WIDE_WQ_ACTIVE)."""
        return self.get_option(INFO_WIDE_WQ_ACTIVE) == 1

    def set_params(self, pi: np.ndarray, A: np.ndarray, B: np.ndarray) -> None:
        pi = np.ascontiguousarray(pi, dtype=np.float64).reshape(self.N)
        A = np.ascontiguousarray(A, dtype=np.float64).reshape(self.N, self.N)
        B = np.ascontiguousarray(B, dtype=np.float64).reshape(self.N, self.M)
        check(self._lib.hmmbw_set_params(self._ctx, pi.ctypes.data, A.ctypes.data, B.ctypes.data))

    @property
    def topology(self) -> str:
        out = ctypes.c_int()
        check(self._lib.hmmbw_get_topology(self._ctx, ctypes.byref(out)))
        return TOPOLOGY_NAME[out.value]

    @property
    def stats_len(self) -> int:
        n = ctypes.c_int64()
        check(self._lib.hmmbw_stats_len(self._ctx, ctypes.byref(n)))
        return n.value

    # -------------------------------------------------------------------------------- training
    def reset(self, epsilon: float, max_iterations: int) -> None:
        check(self._lib.hmmbw_reset_training(self._ctx, float(epsilon), int(max_iterations)))

    def status(self, first: int = 0, count: int = 0) -> Tuple[Status, List[Tuple[float, float]]]:
        st = Status()
        recs = (IterRecord * max(count, 1))()
        check(self._lib.hmmbw_get_status(self._ctx, ctypes.byref(st), ctypes.cast(recs, ctypes.c_void_p) if count
                                         else None, int(first), int(count)))
        return st, [(recs[i].log_likelihood, recs[i].diff) for i in range(count)]

    def enqueue_iterations(self, n: int, stats: Optional[torch.Tensor] = None, group=None) -> None:
        """Enqueue n EM iterations (asynchronous).  Multi-rank when world_size > 1."""
        if self.world_size == 1 or self._native:
            check(self._lib.hmmbw_iterate(self._ctx, int(n)))
            return
        import torch.distributed as dist
        ptr = ctypes.c_void_p(stats.data_ptr())
        for _ in range(int(n)):
            check(self._lib.hmmbw_estep(self._ctx, ptr))
            dist.all_reduce(stats, group=group)  # ONE RCCL all-reduce of the packed fp64 statistics
            check(self._lib.hmmbw_mstep(self._ctx, ptr, self.n_seq_global))

    def iterate_begin(self, n_seq_global: Optional[int] = None) -> Tuple[int, int]:
        """First half of one multi-rank EM iteration (hmmbw_iterate_begin): enqueue this rank's E-step
        and return (device pointer, doubles) of the buffer every rank must all-reduce (sum, in place)
        before iterate_end().  The same enqueue sequence hmmbw_iterate runs around ncclAllReduce."""
        ptr = ctypes.c_void_p()
        n = ctypes.c_int64()
        R = self.n_seq_global if n_seq_global is None else int(n_seq_global)
        check(self._lib.hmmbw_iterate_begin(self._ctx, R, ctypes.byref(ptr), ctypes.byref(n)))
        return int(ptr.value or 0), int(n.value)

    def iterate_end(self) -> None:
        """Second half: the M-step + convergence step from the all-reduced buffer (hmmbw_iterate_end)."""
        check(self._lib.hmmbw_iterate_end(self._ctx))

    def make_stats_buffer(self) -> torch.Tensor:
        return torch.zeros(self.stats_len, dtype=torch.float64, device=f"cuda:{self.device}")

    def train(self, epsilon: float = 1e-6, max_iterations: int = 100, on_iteration: Optional[IterCallback] = None,
              group=None, max_chunk: int = 32, metrics: Optional[str] = None) -> Status:
        """Run EM to the reference's stop rule; on_iteration(k, L_k, diff_k) for every iteration.

        metrics (or the HMMBW_METRICS environment variable): a JSONL file that rank 0 appends one line
        per EM iteration to (see _write_metrics)."""
        self.reset(epsilon, max_iterations)
        stats = self.make_stats_buffer() if self.world_size > 1 and not self._native else None
        mpath = metrics if metrics is not None else os.environ.get("HMMBW_METRICS")
        mfh = open(mpath, "a") if (mpath and self.rank == 0) else None
        timing_prev = self._timing_mode
        if mfh is not None:
            # metrics need the E-step kernel time: events around every launch unless the caller already
            # samples (then its mode and accumulation are left alone; rows use deltas).  Events on every
            # launch serialise the queue around them, so ms_per_iter reads a few us high in this mode.
            if timing_prev == 0:
                self.timing(1)
            self._mbase = (*self.timing(-1), *self.comm_info()[1:])
        # Pipelined: chunk k + 1 is queued before chunk k's status snapshot is read (hmmbw_status_post
        # / _wait wait for the snapshot only), so the device never idles on a host round trip.  The
        # snapshots lag one iteration (the last iteration's M-step is merged into the next launch);
        # iterations queued past the stop rule are device-side no-ops, and the final synchronous
        # status covers the rest.  Every rank takes the same decisions (identical device states).
        max_it = int(max_iterations)
        reported, chunk, queued = 0, 1, 0
        inflight = collections.deque()  # (ticket, iterations queued up to it)
        t_last = time.perf_counter()
        st = None
        try:
            while True:
                if queued < max_it:
                    n = min(chunk, max_it - queued)
                    self.enqueue_iterations(n, stats, group)
                    queued += n
                    chunk = min(chunk * 2, max_chunk)
                    tk = ctypes.c_int64()
                    check(self._lib.hmmbw_status_post(self._ctx, reported, ctypes.byref(tk)))
                    inflight.append((tk.value, queued))
                if not inflight:
                    break
                if len(inflight) < 2 and queued < max_it:
                    continue  # keep two snapshots' worth of work queued
                ticket, upto = inflight.popleft()
                st, recs = self._wait_status(ticket, reported)
                now = time.perf_counter()
                new = st.iterations - reported
                if on_iteration is not None:
                    for k, (L, d) in enumerate(recs):
                        on_iteration(reported + k, L, d)
                if mfh is not None and new > 0:
                    self._write_metrics(mfh, reported, recs, now - t_last, new)
                t_last = now
                reported = st.iterations
                if st.done:
                    break
            st, recs = self.status(reported, 0)  # synchronous: flushes the pending M-step
            new = st.iterations - reported
            if new > 0:
                recs = self.status(reported, new)[1]
                if on_iteration is not None:
                    for k, (L, d) in enumerate(recs):
                        on_iteration(reported + k, L, d)
                if mfh is not None:
                    self._write_metrics(mfh, reported, recs, time.perf_counter() - t_last, new)
        finally:
            if mfh is not None:
                if timing_prev == 0:
                    self.timing(0)
                mfh.close()
        return st

    def post_status(self, first: int = 0) -> int:
        """Enqueue a status snapshot (hmmbw_status_post: no M-step flush, the records of every iteration
        enqueued so far but the last, whose M-step is merged into the next launch) and return its ticket."""
        tk = ctypes.c_int64()
        check(self._lib.hmmbw_status_post(self._ctx, int(first), ctypes.byref(tk)))
        return tk.value

    def live_status(self, on: bool = True) -> None:
        """HMMBW_OPT_LIVE_STATUS: the M-steps mirror every iteration record into pinned host memory, which
        wait_live() polls (synchronises the engine stream once, when switched)."""
        check(self._lib.hmmbw_set_option(self._ctx, OPT_LIVE_STATUS, 1 if on else 0))

    def wait_live(self, iterations: int, first: int = 0,
                  count: int = 0) -> Tuple[Status, List[Tuple[float, float]]]:
        """Wait (polling the host mirror, no stream sync) until `iterations` EM iterations are recorded or EM
        stopped; status + the records [first, first+count)."""
        st = Status()
        recs = (IterRecord * max(count, 1))()
        check(self._lib.hmmbw_status_live_wait(self._ctx, int(iterations), ctypes.byref(st),
                                               ctypes.cast(recs, ctypes.c_void_p) if count else None,
                                               int(first), int(count)))
        return st, [(recs[i].log_likelihood, recs[i].diff) for i in range(count)]

    def wait_status(self, ticket: int, first: int = 0) -> Tuple[Status, List[Tuple[float, float]]]:
        """Wait for snapshot `ticket` only (not for the work queued after it): status + records [first, ...)."""
        return self._wait_status(ticket, first)

    def _wait_status(self, ticket: int, first: int) -> Tuple[Status, List[Tuple[float, float]]]:
        """Status snapshot `ticket` (hmmbw_status_wait) with the records of iterations [first, ...)."""
        st = Status()
        check(self._lib.hmmbw_status_wait(self._ctx, int(ticket), ctypes.byref(st), None, 0, 0))
        count = int(st.iterations) - int(first)
        if count <= 0:
            return st, []
        recs = (IterRecord * count)()
        check(self._lib.hmmbw_status_wait(self._ctx, int(ticket), ctypes.byref(st),
                                          ctypes.cast(recs, ctypes.c_void_p), int(first), count))
        return st, [(recs[i].log_likelihood, recs[i].diff) for i in range(count)]

    def _write_metrics(self, fh, first: int, recs, wall_s: float, enqueued: int) -> None:
        """One JSON line per iteration of the chunk: L and diff (hmm_training.py:503-514), the chunk's
        wall time per enqueued iteration (incl. the host status sync), utterances/s/iter over all ranks,
        the mean E-step kernel time (HIP events), the SURVEY §8(d) byte model over it as GB/s and as a
        fraction of the 8 TB/s HBM peak, and the mean RCCL all-reduce time (engine communicator)."""
        k_ms1, k_n1 = self.timing(-1)  # query only: deltas since the previous row
        _, ar_ms1, ar_n1 = self.comm_info()
        k_ms0, k_n0, ar_ms0, ar_n0 = self._mbase
        self._mbase = (k_ms1, k_n1, ar_ms1, ar_n1)
        k_ms, k_n, ar_ms, ar_n = k_ms1 - k_ms0, k_n1 - k_n0, ar_ms1 - ar_ms0, ar_n1 - ar_n0
        estep_s = k_ms / k_n / 1e3 if k_n else None
        nbytes = 24 * self.n_symbols_total + 16 * self.N * self.n_symbols_total + 8 * self.n_seq
        per_iter = wall_s / max(enqueued, 1)
        for k, (L, d) in enumerate(recs):
            row = {"iteration": first + k + 1, "log_likelihood": L, "diff": d if d != float("inf") else None,
                   "ms_per_iter": 1e3 * per_iter, "utt_per_s_iter": self.n_seq_global / per_iter,
                   "estep_us": 1e6 * estep_s if estep_s else None,
                   "hbm_model_gbs": nbytes / estep_s / 1e9 if estep_s else None,
                   "roofline_frac": nbytes / estep_s / 8e12 if estep_s else None,
                   "allreduce_us": 1e3 * ar_ms / ar_n if ar_n else None,
                   "ranks": self.world_size, "sequences_global": self.n_seq_global}
            fh.write(json.dumps(row) + "\n")
        fh.flush()

    # -------------------------------------------------------------------------------- results
    def params(self, normalise: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        pi = np.zeros(self.N)
        A = np.zeros((self.N, self.N))
        B = np.zeros((self.N, self.M))
        check(self._lib.hmmbw_get_params(self._ctx, pi.ctypes.data, A.ctypes.data, B.ctypes.data, int(normalise)))
        return pi, A, B

    def loglik(self) -> np.ndarray:
        out = np.zeros(max(self.n_seq, 1))
        check(self._lib.hmmbw_get_loglik(self._ctx, out.ctypes.data))
        return out[: self.n_seq]

    def score(self) -> np.ndarray:
        """Forward-only log P(O_r | lambda) of every loaded sequence (hmm_testing.py:49-104)."""
        out = np.zeros(max(self.n_seq, 1))
        check(self._lib.hmmbw_score(self._ctx, out.ctypes.data))
        return out[: self.n_seq]

    def timing(self, enable: int = -1) -> Tuple[float, int]:
        """(accumulated E-step ms, timed launches) of hmmbw_timing; enable >= 0 also resets and sets the
        mode (0 off, k: every k-th launch), enable < 0 only queries."""
        if enable >= 0:
            self._timing_mode = int(enable)
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._lib.hmmbw_timing(self._ctx, int(enable), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def timing_split(self) -> Tuple[float, int]:
        """(E-step kernel ms, count) of the timed launches that run a follow-up kernel after the E-step
        kernel (wide path: k_bnum_gather) -- hmmbw_timing_split; same reset as timing()."""
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._lib.hmmbw_timing_split(self._ctx, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def comm_info(self, reset: bool = False) -> Tuple[int, float, int]:
        """(ranks of the engine's RCCL communicator (0: none), all-reduce ms summed over the timed
        iterations, number of timed all-reduces) -- hmmbw_comm_info."""
        n = ctypes.c_int()
        ms = ctypes.c_double()
        cnt = ctypes.c_int64()
        check(self._lib.hmmbw_comm_info(self._ctx, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(cnt), int(reset)))
        return n.value, ms.value, cnt.value

    def comm_payload_bytes(self) -> int:
        """Bytes of the last all-reduce hmmbw_iterate enqueued on the engine communicator (0: none)."""
        n = ctypes.c_int64()
        check(self._lib.hmmbw_comm_payload(self._ctx, ctypes.byref(n)))
        return 8 * n.value

    def close(self, timeout_s: Optional[float] = None) -> None:
        """Destroy the context.  With the peer all-reduce set up, every rank should call close() at the same
        point: the ranks first meet (a bounded rendezvous on the process group's store, HMMBW_CLOSE_TIMEOUT_S,
        default 60 s), so no rank frees its IPC-exported receive region while another may still push into it
        (a rank whose wait timed out, or bench's fallback after a failed leg).  A rank that closes alone (an
        exception path) is not held forever: after the timeout it frees its context anyway, and the ranks
        still iterating then stop on their own bounded peer wait (HMMBW_E_TIMEOUT)."""
        if getattr(self, "_ctx", None):
            if getattr(self, "_peer_ok", False) and self.world_size > 1:
                try:
                    import torch.distributed as dist
                    if dist.is_available() and dist.is_initialized():
                        torch.cuda.synchronize(self.device)  # this rank's pushes have landed
                        if timeout_s is None:
                            timeout_s = float(os.environ.get("HMMBW_CLOSE_TIMEOUT_S", "60"))
                        self._close_rendezvous(timeout_s)    # ... and every other rank's too (bounded)
                except Exception:  # noqa: BLE001 - a broken process group must not keep the context alive
                    pass
            self._lib.hmmbw_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            if getattr(self, "_ctx", None):  # garbage collection is no collective: skip the barrier
                self._peer_ok = False
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class EngineGroup:
    """Several single-rank engines of one shape (same N, M, resolved topology, device and stream),
    advanced by ONE grouped E-step launch per EM iteration and scored by one launch (hmmbw_group_*).

    Replaces the per-word training loop of HMM/main.py:147-152 and the per-(recording, model) scoring
    loop of HMM/hmm_testing.py:139-161.  Every member keeps its own parameters, statistics and stop
    rule (hmm_training.py:346), so each ends exactly where training it alone would."""

    def __init__(self, engines: Sequence[BaumWelchEngine]):
        self._lib = lib()
        self.engines = list(engines)
        n = len(self.engines)
        arr = (ctypes.c_void_p * max(n, 1))(*[e._ctx.value for e in self.engines])
        g = ctypes.c_void_p()
        check(self._lib.hmmbw_group_create(arr, n, ctypes.byref(g)))
        self._g = g

    def enqueue_iterations(self, n: int) -> None:
        check(self._lib.hmmbw_group_iterate(self._g, int(n)))

    def train(self, epsilon: float = 1e-6, max_iterations: int = 100,
              on_iteration: Optional[Callable[[int, int, float, float], None]] = None,
              max_chunk: int = 32) -> List[Status]:
        """EM on every member to its own stop rule; on_iteration(member, k, L_k, diff_k)."""
        for e in self.engines:
            e.reset(epsilon, max_iterations)
        reported = [0] * len(self.engines)
        chunk = 1
        while True:
            sts = [e.status()[0] for e in self.engines]
            live = [s for s in sts if not s.done]
            if not live:
                break
            n = max(1, min(chunk, int(max_iterations) - min(s.iterations for s in live)))
            self.enqueue_iterations(n)
            for i, e in enumerate(self.engines):
                st, _ = e.status()
                if on_iteration is not None and st.iterations > reported[i]:
                    st, recs = e.status(reported[i], st.iterations - reported[i])
                    for k, (L, d) in enumerate(recs):
                        on_iteration(i, reported[i] + k, L, d)
                reported[i] = st.iterations
            chunk = min(chunk * 2, max_chunk)
        return [e.status()[0] for e in self.engines]

    def score(self) -> List[np.ndarray]:
        """Forward-only log P(O_r | lambda_m) of every member's sequences, one launch."""
        total = sum(e.n_seq for e in self.engines)
        out = np.zeros(max(total, 1))
        check(self._lib.hmmbw_group_score(self._g, out.ctypes.data))
        res, off = [], 0
        for e in self.engines:
            res.append(out[off: off + e.n_seq].copy())
            off += e.n_seq
        return res

    def timing(self, enable: int = -1) -> Tuple[float, int]:
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._lib.hmmbw_group_timing(self._g, int(enable), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def close(self) -> None:
        if getattr(self, "_g", None):
            self._lib.hmmbw_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
