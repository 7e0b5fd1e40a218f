"""Drop-in for HMM/hmm_training.py of DemianMArin/HMM_Training, backed by the MI355X engine.

Same names, signatures, printed lines, return order and error behaviour as the reference:

* ``hmm_training(observations, N=4, M=256, epsilon=1e-6, max_iterations=100, show_progress=True,
  word_name=None, load_initial_params=True) -> (A, B, pi)``            (hmm_training.py:265-541)
* ``training_with_save(word_recordings, centroids, word_name, ...) -> HMMTrained`` (:215-247)
* ``get_observations(recordings, centroids)``                            (:82-120, HIP encoder)
* ``safe_log`` / ``safe_exp`` / ``log_sum_exp``                          (:46-79)

The EM iterations run in hand-written HIP kernels (hmm_training_amd/csrc/hmmbw.hip) through the C
ABI of include/hmmbw.h.  When ``torch.distributed`` is initialised with world_size > 1, every rank
calls ``hmm_training`` with the same list, trains on its contiguous length-balanced shard, and
all ranks return identical parameters (one RCCL all-reduce of the statistics per iteration).
"""
from __future__ import annotations

import json
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .engine import BaumWelchEngine, shard_bounds
from .hmm_classes import DataStorageHMM, HMMTrained

WARM_START_DIR = "../Data/Eighty-five-percent_20"  # hmm_training.py:278


def safe_log(x):
    """log x, -inf where x <= 0 (hmm_training.py:46-54)."""
    if isinstance(x, np.ndarray):
        out = np.full_like(x, -np.inf, dtype=float)
        pos = x > 0
        out[pos] = np.log(x[pos])
        return out
    return math.log(x) if x > 0 else float("-inf")


def safe_exp(x):
    """exp x, 0 where x == -inf (hmm_training.py:56-64)."""
    if isinstance(x, np.ndarray):
        out = np.zeros_like(x, dtype=float)
        fin = x != -np.inf
        out[fin] = np.exp(x[fin])
        return out
    return math.exp(x) if x != float("-inf") else 0.0


def log_sum_exp(log_probs):
    """log sum exp over the finite entries; -inf if none; scalars pass through (:66-79)."""
    if isinstance(log_probs, np.ndarray):
        fin = log_probs[log_probs != -np.inf]
        if fin.size == 0:
            return float("-inf")
        top = np.max(fin)
        return top + math.log(np.sum(np.exp(fin - top)))
    return log_probs if log_probs != float("-inf") else float("-inf")


def get_observations(recordings, centroids, device: Optional[int] = None) -> List[np.ndarray]:
    """Vector quantisation (hmm_training.py:82-120): per frame, the index of the nearest centroid by
    Euclidean distance over mfcc[1:] (power coefficient excluded), first minimum on ties.  All frames
    of all recordings go through ONE launch of the HIP encoder (hmmbw_vq_encode), whose distances are
    computed exactly as np.linalg.norm does, so the indices are the reference's bit for bit."""
    if len(centroids) == 0:
        return [np.zeros(len(r), dtype=np.int64) for r in recordings]
    C = np.stack([np.asarray(c.mfcc, dtype=np.float64).reshape(-1) for c in centroids])
    lengths = [len(r) for r in recordings]
    frames = [np.asarray(f.mfcc, dtype=np.float64).reshape(-1) for rec in recordings for f in rec]
    if not frames:
        return [np.array([]) for _ in recordings]
    Fm = np.stack(frames)
    if Fm.shape[1] != C.shape[1]:
        raise ValueError(f"operands could not be broadcast together with shapes ({Fm.shape[1] - 1},) "
                         f"({C.shape[1] - 1},)")
    symbols = vq_encode(Fm, C, device=device)
    out, pos = [], 0
    for T in lengths:
        out.append(symbols[pos:pos + T].astype(np.int64) if T else np.array([]))
        pos += T
    return out


def vq_encode(frames: np.ndarray, centroids: np.ndarray, device: Optional[int] = None, first_dim: int = 1,
              return_distances: bool = False):
    """[F] nearest-centroid indices (int64) of frames [F][D] against centroids [K][D] over the columns
    [first_dim, D) on the GPU (hmmbw_vq_encode, include/hmmbw.h)."""
    import ctypes

    import torch

    from ._lib import check, lib
    frames = np.ascontiguousarray(frames, dtype=np.float64)
    centroids = np.ascontiguousarray(centroids, dtype=np.float64)
    F, D = frames.shape
    K = centroids.shape[0]
    dims = D - first_dim
    if F == 0:
        return (np.zeros(0, np.int64), np.zeros(0)) if return_distances else np.zeros(0, np.int64)
    if dims <= 0:  # every distance is norm([]) = 0: the first centroid wins
        z = np.zeros(F, dtype=np.int64)
        return (z, np.zeros(F)) if return_distances else z
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
    L = lib()
    with torch.cuda.device(dev):
        tf = torch.from_numpy(frames).to(dev)
        tc = torch.from_numpy(centroids).to(dev)
        ts = torch.empty(F, dtype=torch.int32, device=dev)
        td = torch.empty(F, dtype=torch.float64, device=dev) if return_distances else None
        stream = torch.cuda.current_stream(dev).cuda_stream
        check(L.hmmbw_vq_encode(ctypes.c_void_p(stream), ctypes.c_void_p(tf.data_ptr()), F, D, first_dim, dims,
                                ctypes.c_void_p(tc.data_ptr()), K, ctypes.c_void_p(ts.data_ptr()),
                                ctypes.c_void_p(td.data_ptr()) if td is not None else None))
        sym = ts.cpu().numpy().astype(np.int64)
        if return_distances:
            return sym, td.cpu().numpy()
    return sym


def default_initial_params(N: int, M: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The reference's defaults (hmm_training.py:300-318).  They are hard-coded 4-state arrays, so
    for N < 4 the reference reads their leading N entries (reproduced here); for N > 4 it raises
    IndexError at :360, and this build uses its own left-to-right generalisation instead:
    pi = [0.97, 0.03/(N-1), ...], a_ii = 0.6, a_i,i+1 = 0.4, absorbing last state, B = 1/M."""
    if N <= 4:
        pi = np.array([0.97, 0.02, 0.005, 0.005])[:N].copy()
        A = np.array([[0.6, 0.4, 0.0, 0.0], [0.0, 0.6, 0.4, 0.0], [0.0, 0.0, 0.6, 0.4],
                      [0.0, 0.0, 0.0, 1.0]])[:N, :N].copy()
    else:
        pi = np.full(N, 0.03 / (N - 1))
        pi[0] = 0.97
        A = np.zeros((N, N))
        idx = np.arange(N - 1)
        A[idx, idx] = 0.6
        A[idx, idx + 1] = 0.4
        A[N - 1, N - 1] = 1.0
    B = np.full((N, M), 1.0 / M)
    return pi, A, B


def _load_warm_start(word_name: str, N: int, M: int, show_progress: bool):
    """hmm_training.py:275-297 (same messages, same swallowed errors)."""
    try:
        saved = DataStorageHMM.load_hmm(word_name, WARM_START_DIR)
        if saved.states == N and saved.symbols == M:
            if show_progress:
                print(f"Loaded initial parameters from saved model for word '{word_name}'")
            return saved.Pi.copy(), saved.A.copy(), saved.B.copy()
        if show_progress:
            print(f"Saved model dimensions ({saved.states} states, {saved.symbols} symbols) "
                  f"don't match expected ({N} states, {M} symbols). Using default initialization.")
    except (FileNotFoundError, json.JSONDecodeError, KeyError) as exc:
        if show_progress:
            print(f"Could not load saved model for word '{word_name}': {str(exc)}. Using default initialization.")
    except Exception as exc:
        if show_progress:
            print(f"Unexpected error loading saved model for word '{word_name}': {str(exc)}. "
                  "Using default initialization.")
    return None


def _dist_context(group=None):
    try:
        import torch.distributed as dist
    except ImportError:
        return 0, 1, None
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group), group
    return 0, 1, None


def _initial_params(N: int, M: int, word_name, load_initial_params: bool, show_progress):
    """Warm start or defaults, with the reference's messages (hmm_training.py:270-325)."""
    pi0 = A0 = B0 = None
    if load_initial_params and word_name:
        loaded = _load_warm_start(word_name, N, M, show_progress)
        if loaded is not None:
            pi0, A0, B0 = loaded
    dpi, dA, dB = default_initial_params(N, M)
    if pi0 is None:
        pi0 = dpi
        if show_progress:
            print("Using default initial state probabilities")
    if A0 is None:
        A0 = dA
        if show_progress:
            print("Using default transition matrix")
    if B0 is None:
        B0 = dB
        if show_progress:
            print("Using default emission matrix")
    return pi0, A0, B0


def _final_lines(st, max_iterations: int) -> None:
    """The closing lines of hmm_training.py:516-521 (and its unbound-local error when no iteration ran)."""
    if st.iterations == 0:
        # the reference's while-loop never ran: :517 reads an unbound local
        raise UnboundLocalError("local variable 'current_log_likelihood_sum' referenced before assignment")
    L, diff = st.last_log_likelihood, st.last_diff
    print(f"Log-likelihood: {L:.6f}, Diff: {diff:.8f}")
    if st.iterations >= max_iterations:
        print(f"Reached maximum iterations ({max_iterations})")
    else:
        print(f"Converged after {st.iterations} iterations")


def hmm_training(observations: List[np.ndarray], N: int = 4, M: int = 256, epsilon: float = 1e-6,
                 max_iterations: int = 100, show_progress=True, word_name: str = None,
                 load_initial_params: bool = True, *, device: Optional[int] = None, topology: str = "auto",
                 group=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Baum-Welch EM for one discrete HMM; returns (A, B, pi) like hmm_training.py:265-541.

    Under torch.distributed (world_size > 1) only rank 0 prints the reference's progress lines, so
    a torchrun of the drop-in shows them once; every rank returns the same parameters."""
    rank, world, group = _dist_context(group)
    if rank != 0:
        show_progress = False
    pi0, A0, B0 = _initial_params(N, M, word_name, load_initial_params, show_progress)
    obs = list(observations)
    if world > 1:
        lo, hi = shard_bounds([len(o) for o in obs], world)[rank]
        local = obs[lo:hi]
        if device is None:
            import torch
            device = int(os.environ.get("LOCAL_RANK", rank)) % max(torch.cuda.device_count(), 1)
    else:
        local = obs

    engine = BaumWelchEngine(N, M, device=device, topology=topology, rank=rank, world_size=world, group=group)
    try:
        engine.set_observations(local, n_seq_global=len(obs))
        engine.set_params(pi0, A0, B0)

        def report(k: int, L: float, diff: float) -> None:
            if show_progress:
                print(f"Iteration {k + 1}")
                print(f"Log-likelihood: {L:.6f}, Diff: {diff:.8f}")

        st = engine.train(epsilon, max_iterations, report, group=group)
        if st.iterations == 0:
            # the reference's while-loop never ran: :517 reads an unbound local
            raise UnboundLocalError("local variable 'current_log_likelihood_sum' referenced before assignment")
        if rank == 0:
            _final_lines(st, max_iterations)
        pi, A, B = engine.params(normalise=True)
    finally:
        engine.close()
    return A, B, pi


def hmm_training_group(observation_sets: Sequence[List[np.ndarray]], N: int = 4, M: int = 256,
                       epsilon: float = 1e-6, max_iterations: int = 100, show_progress=True,
                       word_names: Optional[Sequence[Optional[str]]] = None, load_initial_params: bool = True, *,
                       device: Optional[int] = None, topology: str = "auto",
                       stdout_parts: Optional[List[str]] = None) -> List[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
    """``hmm_training`` for several word models at once (the loop of HMM/main.py:147-152).

    The models of one shape train together: ONE grouped E-step launch per EM iteration
    (hmmbw_group_iterate) instead of one training run per word.  Each model keeps its own stop rule,
    so every returned (A, B, pi) equals what ``hmm_training`` returns for that word alone.  The
    printed lines are each word's own, in word order, as if the words had been trained one after
    another; with ``stdout_parts`` they are returned per word instead of printed.  Models that
    cannot be grouped (N > 16, tables too large for LDS, several ranks) train one by one."""
    import contextlib
    import io

    from .engine import EngineGroup

    n = len(observation_sets)
    names = list(word_names) if word_names is not None else [None] * n
    bufs = [io.StringIO() for _ in range(n)]
    rank, world, _ = _dist_context(None)
    if world > 1:  # data-parallel ranks: each word's run is itself sharded (hmm_training)
        out = []
        for i, obs in enumerate(observation_sets):
            with contextlib.redirect_stdout(bufs[i]):
                out.append(hmm_training(obs, N, M, epsilon, max_iterations, show_progress, names[i],
                                        load_initial_params, device=device, topology=topology))
        if stdout_parts is not None:
            stdout_parts.extend(b.getvalue() for b in bufs)
        else:
            for b in bufs:
                print(b.getvalue(), end="")
        return out
    engines: List[Optional[BaumWelchEngine]] = [None] * n
    results: List[Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]]] = [None] * n
    try:
        for i, obs in enumerate(observation_sets):
            with contextlib.redirect_stdout(bufs[i]):
                pi0, A0, B0 = _initial_params(N, M, names[i], load_initial_params, show_progress)
            eng = BaumWelchEngine(N, M, device=device, topology=topology)
            engines[i] = eng
            eng.set_observations(list(obs))
            eng.set_params(pi0, A0, B0)
        groupable = N <= 16
        buckets = {}
        for i, eng in enumerate(engines):
            buckets.setdefault(eng.topology if groupable else i, []).append(i)
        statuses = [None] * n
        for members in buckets.values():
            def report(m: int, k: int, L: float, diff: float, members=members) -> None:
                if show_progress:
                    bufs[members[m]].write(f"Iteration {k + 1}\nLog-likelihood: {L:.6f}, Diff: {diff:.8f}\n")
            try:
                grp = EngineGroup([engines[i] for i in members])
            except Exception:  # shape the grouped kernel does not take: train one by one
                grp = None
            if grp is not None:
                with grp:
                    sts = grp.train(epsilon, max_iterations, report)
            else:
                sts = []
                for m, i in enumerate(members):
                    sts.append(engines[i].train(epsilon, max_iterations,
                                                lambda k, L, d, m=m: report(m, k, L, d)))
            for m, i in enumerate(members):
                statuses[i] = sts[m]
        for i, eng in enumerate(engines):
            st = statuses[i]
            with contextlib.redirect_stdout(bufs[i]):
                _final_lines(st, max_iterations)
            pi, A, B = eng.params(normalise=True)
            results[i] = (A, B, pi)
    finally:
        for eng in engines:
            if eng is not None:
                eng.close()
    if stdout_parts is not None:
        stdout_parts.extend(b.getvalue() for b in bufs)
    else:
        for b in bufs:
            print(b.getvalue(), end="")
    return results


def training_with_save(word_recordings, centroids, word_name: str, max_iterations=100, show_progress=True,
                       load_initial_params=False, *, n_states: int = 4, base_dir: Optional[str] = None) -> HMMTrained:
    """VQ -> hmm_training(N=4) -> HMMTrained -> save JSON (hmm_training.py:215-247)."""
    print("Converting recordings to observations...")
    observations = get_observations(word_recordings, centroids)
    print(f"Generated {len(observations)} observation sequences")
    print(f"Sequence lengths: {[len(obs) for obs in observations]}")
    print("Starting Baum-Welch training...")
    A, B, pi = hmm_training(observations, N=n_states, M=len(centroids), max_iterations=max_iterations,
                            show_progress=show_progress, word_name=word_name,
                            load_initial_params=load_initial_params)
    model = HMMTrained(states=n_states, symbols=len(centroids), A=A, B=B, Pi=pi, word=word_name)
    if base_dir is None:
        DataStorageHMM.save_hmm(model, print_messages=False)
    else:
        DataStorageHMM.save_hmm(model, base_dir=base_dir, print_messages=False)
    return model
