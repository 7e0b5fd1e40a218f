"""The multi-rank iteration an RCCL run enqueues, run at world 2/3/5/8 with every rank in this process on
cuda:0.  hmmbw_iterate_begin / hmmbw_iterate_end split hmmbw_iterate at its ncclAllReduce, so each
engine runs exactly the kernels an 8-GPU job runs (on the small kernels: the fused E-step that
accumulates into the all-reduce buffer, the rank's (max, sum exp) pair at slot 2 * rank, the
last-workgroup fold, the empty-shard memset, world-sized LL slots, the merged or standalone M-step on
the all-reduced buffer, small and wide; in deterministic mode: hmmbw_estep + k_reduce_local), and the
test sums the W buffers in between (the all-reduce).

Every rank must end on the reference's (pi, A, B) and L trace for the unsharded data
(hmm_training.py:351-514, :415-424 pi / R over all ranks, :503 L = LSE over all sequences), and all
ranks must hold bitwise-identical L records and parameters (they take the stop decision of :346
independently; ranks with an empty shard run the standalone M-step kernel, the others the merged one).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

PARAM_RTOL, PARAM_ATOL, LL_RTOL = 1e-6, 1e-15, 1e-9


@pytest.fixture(scope="module")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    h = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    h.hipMemcpy.restype = ctypes.c_int
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return h


def load(case):
    return np.load(f"{GOLDEN}/bw_{case}.npz", allow_pickle=False)


def observations(d):
    off, sym = d["offsets"], d["symbols"]
    return [sym[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def assert_params(mine, ref, what):
    err = np.abs(np.asarray(mine) - ref) - (PARAM_RTOL * np.abs(ref) + PARAM_ATOL)
    assert np.all(err <= 0), f"{what}: worst excess {err.max():.3e}"


def allreduce_in_process(hip, bufs):
    """Sum the ranks' device buffers (ptr, n) in place: gather into torch, add in rank order, scatter."""
    import torch
    n = bufs[0][1]
    assert all(b[1] == n for b in bufs), "ranks disagree on the all-reduce length"
    torch.cuda.synchronize()
    tot = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    tmp = torch.empty_like(tot)
    for ptr, _ in bufs:
        assert hip.hipMemcpy(ctypes.c_void_p(tmp.data_ptr()), ctypes.c_void_p(ptr), 8 * n, 3) == 0
        tot += tmp
    torch.cuda.synchronize()
    for ptr, _ in bufs:
        assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(tot.data_ptr()), 8 * n, 3) == 0
    torch.cuda.synchronize()


def run_world(hip, d, world, deterministic=False, copies=None):
    from hmm_training_amd.engine import BaumWelchEngine, shard_bounds
    N, M = int(d["N"]), int(d["M"])
    obs = observations(d)
    bounds = shard_bounds([len(o) for o in obs], world)
    engines = []
    try:
        for r, (lo, hi) in enumerate(bounds):
            e = BaumWelchEngine(N, M, rank=r, world_size=world, deterministic=deterministic, stat_copies=copies)
            e.set_observations(obs[lo:hi], n_seq_global=len(obs))
            e.set_params(d["init_pi"], d["init_A"], d["init_B"])
            e.reset(float(d["epsilon"]), int(d["max_iterations"]))
            engines.append(e)
        # iterations past the stop rule are device-side no-ops on every rank (the reference stops there)
        for _ in range(int(d["max_iterations"]) + 1):
            bufs = [e.iterate_begin() for e in engines]
            allreduce_in_process(hip, bufs)
            for e in engines:
                e.iterate_end()
        out = []
        for e in engines:
            st, recs = e.status(0, int(d["iterations"]))
            out.append((st, recs, e.params(normalise=False), e.params(normalise=True)))
        return bounds, out
    finally:
        for e in engines:
            e.close()


CASES = ["n8_k256_t200", "converge", "zero_prob_seq", "dense_n16", "n64_k1024_tiny", "n5_k256_cfg1"]


@pytest.mark.parametrize("deterministic", [False, True])
@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("case", CASES)
def test_split_iteration_multirank_matches_reference(hip, case, world, deterministic):
    d = load(case)
    bounds, out = run_world(hip, d, world, deterministic)
    for r, (st, recs, raw, (pi, A, B)) in enumerate(out):
        assert st.done and st.iterations == int(d["iterations"]), f"rank {r} ({bounds[r]})"
        L = np.array([x for x, _ in recs])
        np.testing.assert_allclose(L, d["trace_L"], rtol=LL_RTOL)
        assert_params(A, d["out_A"], f"A rank {r}")
        assert_params(B, d["out_B"], f"B rank {r}")
        assert_params(pi, d["out_pi"], f"pi rank {r}")
    # replicated state: every rank bitwise equal to rank 0 (records, diffs, working parameters)
    st0, recs0, raw0, _ = out[0]
    for r, (st, recs, raw, _) in enumerate(out[1:], 1):
        assert recs == recs0, f"rank {r} L/diff records differ from rank 0"
        assert (st.iterations, st.done, st.converged) == (st0.iterations, st0.done, st0.converged)
        for x, y in zip(raw, raw0):
            np.testing.assert_array_equal(x, y)


def test_split_iteration_empty_shards_present(hip):
    """n64_k1024_tiny has 2 sequences: at world 8, six ranks hold empty shards (the memset branch and
    the standalone M-step beside merged ranks)."""
    from hmm_training_amd.engine import shard_bounds
    d = load("n64_k1024_tiny")
    obs = observations(d)
    bounds = shard_bounds([len(o) for o in obs], 8)
    assert sum(1 for lo, hi in bounds if hi == lo) >= 6


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("N,K,topology,R,tmax", [(8, 256, "left_to_right", 2400, 160), (5, 64, "dense", 2400, 160),
                                                 (40, 96, "dense", 700, 100)])
def test_split_iteration_multirank_vs_oracle(hip, oracle_mt, N, K, topology, R, tmax, world):
    """Every rank holds several workgroups (hundreds of sequences per rank): the per-rank last-workgroup fold over
    several workgroups, ranks' pairs at 2 * rank, world-sized LL slots; against the oracle run on the
    unsharded data, 4 EM iterations (the wide N = 40 case: k_estep_mfma + k_bnum_gather into the buffer)."""
    from hmm_training_amd.engine import BaumWelchEngine, shard_bounds, to_csr
    from hmm_training_amd.hmm_training import default_initial_params
    oracle = oracle_mt
    rng = np.random.default_rng(11 * N + world)
    iters = 4
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(20, tmax, size=R)]
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    B = rng.dirichlet(np.full(K, 2.0), size=N)
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    bounds = shard_bounds([len(o) for o in obs], world)
    engines = []
    try:
        for r, (lo, hi) in enumerate(bounds):
            e = BaumWelchEngine(N, K, rank=r, world_size=world, topology=topology)
            e.set_observations(obs[lo:hi], n_seq_global=R)
            e.set_params(pi, A, B)
            e.reset(0.0, iters)
            engines.append(e)
        for _ in range(iters):
            bufs = [e.iterate_begin() for e in engines]
            allreduce_in_process(hip, bufs)
            for e in engines:
                e.iterate_end()
        res = []
        for e in engines:
            st, recs = e.status(0, iters)
            lp = e.loglik()
            res.append((st, recs, e.params(normalise=True), lp))
    finally:
        for e in engines:
            e.close()
    logp = np.concatenate([r[3] for r in res])
    np.testing.assert_allclose(logp, ref.logP, rtol=LL_RTOL)
    for r, (st, recs, (p2, A2, B2), _) in enumerate(res):
        assert st.iterations == iters and st.done
        np.testing.assert_allclose([x for x, _ in recs], ref.trace_L, rtol=LL_RTOL)
        assert recs == res[0][1], f"rank {r} records differ from rank 0"
        assert_params(A2, ref.A, f"A rank {r}")
        assert_params(B2, ref.B, f"B rank {r}")
        assert_params(p2, ref.pi, f"pi rank {r}")


def test_split_iteration_multirank_joined_map_vs_oracle(hip, oracle_mt):
    """Ranks with more sequence groups than SIMDs (9,000 ragged sequences per rank, left-to-right): the
    joined spread map (k_estep_join, 8-wave workgroups) on the fused multi-rank path, whose last workgroup
    folds the pairs of the 256 launched workgroups; 2 ranks against the oracle on the unsharded data."""
    test_split_iteration_multirank_vs_oracle(hip, oracle_mt, 8, 256, "left_to_right", 18_000, 160, 2)


def test_split_iteration_multirank_work_queue_vs_oracle(hip, oracle_mt, monkeypatch):
    """The wide work-queue E-step (more tiles than CUs per rank, HMMBW_WIDE_WQ=1) on the fused
    multi-rank path: the last backward unit folds the ranks' log-likelihood pairs over every tile."""
    import torch
    monkeypatch.setenv("HMMBW_WIDE_WQ", "1")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    test_split_iteration_multirank_vs_oracle(hip, oracle_mt, 40, 96, "dense", 2 * 16 * (ncu + 9), 40, 2)


def test_split_iteration_stat_copies_and_payload(hip):
    """Fused payload = copies * statistics + one pair per rank, 256-B aligned, identical on every rank."""
    d = load("n8_k256_t200")
    for copies in (1, 3):
        _, out = run_world(hip, d, 3, copies=copies)
        for st, recs, raw, (pi, A, B) in out:
            assert st.iterations == int(d["iterations"])
            assert_params(A, d["out_A"], "A")
            assert_params(B, d["out_B"], "B")


def test_split_iteration_call_order(hip):
    from hmm_training_amd._lib import HMMBW_E_STATE
    from hmm_training_amd.engine import BaumWelchEngine
    d = load("n8_k256_t200")
    with BaumWelchEngine(int(d["N"]), int(d["M"]), rank=0, world_size=2) as e:
        e.set_observations(observations(d)[:5], n_seq_global=10)
        e.set_params(d["init_pi"], d["init_A"], d["init_B"])
        e.reset(1e-6, 3)
        assert e._lib.hmmbw_iterate_end(e._ctx) == HMMBW_E_STATE
        ptr, n = e.iterate_begin()
        assert ptr and n > 0
        p2, n2 = ctypes.c_void_p(), ctypes.c_int64()
        assert e._lib.hmmbw_iterate_begin(e._ctx, 10, ctypes.byref(p2), ctypes.byref(n2)) == HMMBW_E_STATE
        assert e._lib.hmmbw_iterate(e._ctx, 1) == HMMBW_E_STATE
        assert e._lib.hmmbw_reset_training(e._ctx, 1e-6, 3) == HMMBW_E_STATE
        e.iterate_end()


def test_split_iteration_multirank_work_queue_timeout_then_oracle(hip, oracle_mt):
    """a work-queue timeout on the fused multi-rank path leaves the completion counter (the
    last-workgroup fold of the ranks' log-likelihood pairs) part-way, because workgroups that start after the
    stop return before counting.  hmmbw_reset_training clears it: a first run with a 0-ms bound fails with
    HMMBW_E_TIMEOUT on both ranks, then a second run of the same contexts with the default bound must match
    the oracle on the unsharded data (hmm_training.py:351-514, :503 L over all sequences)."""
    import torch
    from hmm_training_amd._lib import HMMBW_E_TIMEOUT, HMMBWError
    from hmm_training_amd.engine import BaumWelchEngine, shard_bounds, to_csr
    from hmm_training_amd.hmm_training import default_initial_params
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    N, K, world, iters = 32, 64, 2, 3
    R = 2 * (16 * ncu + 16 * 9 + 3)
    rng = np.random.default_rng(91)
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(8, 24, size=R)]
    pi, A, B = default_initial_params(N, K)
    A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    B = rng.dirichlet(np.full(K, 2.0), size=N)
    off, sym = to_csr(obs)
    ref = oracle_mt.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    bounds = shard_bounds([len(o) for o in obs], world)
    engines = []
    try:
        for r, (lo, hi) in enumerate(bounds):
            e = BaumWelchEngine(N, K, rank=r, world_size=world, topology="dense")
            e.set_observations(obs[lo:hi], n_seq_global=R)
            e.set_params(pi, A, B)
            e.set_work_queue(1, timeout_ms=0)
            assert e.work_queue_active
            e.reset(0.0, iters)
            engines.append(e)
        for _ in range(iters):
            bufs = [e.iterate_begin() for e in engines]
            allreduce_in_process(hip, bufs)
            for e in engines:
                e.iterate_end()
        for e in engines:
            with pytest.raises(HMMBWError) as ei:
                e.status()
            assert ei.value.code == HMMBW_E_TIMEOUT
        for e in engines:
            e.set_params(pi, A, B)
            e.set_work_queue(1, timeout_ms=10000)
            e.reset(0.0, iters)
        for _ in range(iters):
            bufs = [e.iterate_begin() for e in engines]
            allreduce_in_process(hip, bufs)
            for e in engines:
                e.iterate_end()
        res = []
        for e in engines:
            st, recs = e.status(0, iters)
            res.append((st, recs, e.params(normalise=True), e.loglik()))
    finally:
        for e in engines:
            e.close()
    np.testing.assert_allclose(np.concatenate([r[3] for r in res]), ref.logP, rtol=LL_RTOL)
    for r, (st, recs, (p2, A2, B2), _) in enumerate(res):
        assert st.iterations == iters and st.done
        np.testing.assert_allclose([x for x, _ in recs], ref.trace_L, rtol=LL_RTOL)
        assert_params(A2, ref.A, f"A rank {r}")
        assert_params(B2, ref.B, f"B rank {r}")
        assert_params(p2, ref.pi, f"pi rank {r}")
