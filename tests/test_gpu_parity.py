"""GPU parity: the HIP engine (through the C ABI) against the reference's golden vectors and the
oracle restatement.  Run on an MI355X with `pytest -m gpu`.

Tolerance (north_star: "within 1e-6 relative"): parameters |x - ref| <= 1e-6 * |ref| + 1e-15.  The
absolute 1e-15 term covers entries the reference's safe_exp underflows to exactly 0.0
or leaves at ~1e-300, which the scaled-linear fp64 engine holds as ~1e-300 or at the 1e-20 floor.
Log-likelihoods: relative 1e-9.
"""
import contextlib
import io
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden_cases

pytestmark = pytest.mark.gpu

PARAM_RTOL, PARAM_ATOL, LL_RTOL = 1e-6, 1e-15, 1e-9


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    from hmm_training_amd import _lib
    _lib.lib()


def load(case):
    return np.load(f"{GOLDEN}/bw_{case}.npz", allow_pickle=False)


def observations(d):
    off, sym = d["offsets"], d["symbols"]
    return [sym[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def assert_params(mine, ref, what):
    mine, ref = np.asarray(mine), np.asarray(ref)
    err = np.abs(mine - ref) - (PARAM_RTOL * np.abs(ref) + PARAM_ATOL)
    assert np.all(err <= 0), f"{what}: worst excess {err.max():.3e} at {np.unravel_index(np.argmax(err), err.shape)}"


def assert_ll(mine, ref, rtol=LL_RTOL):
    mine, ref = np.asarray(mine, dtype=float), np.asarray(ref, dtype=float)
    assert np.array_equal(np.isneginf(mine), np.isneginf(ref))
    f = np.isfinite(ref)
    np.testing.assert_allclose(mine[f], ref[f], rtol=rtol)


def run_dropin(d, tmp_path, monkeypatch, **kw):
    """Call the drop-in hmm_training exactly as the reference was called for this fixture."""
    from hmm_training_amd.hmm_classes import DataStorageHMM, HMMTrained
    from hmm_training_amd.hmm_training import hmm_training
    N, M = int(d["N"]), int(d["M"])
    warm = bool(d["load_initial"])
    os.makedirs(tmp_path / "cwd", exist_ok=True)
    if warm:
        DataStorageHMM.save_hmm(HMMTrained(N, M, d["init_A"], d["init_B"], d["init_pi"], "w"),
                                base_dir=str(tmp_path / "Data" / "Eighty-five-percent_20"), print_messages=False)
    monkeypatch.chdir(tmp_path / "cwd")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        A, B, pi = hmm_training(observations(d), N=N, M=M, epsilon=float(d["epsilon"]),
                                max_iterations=int(d["max_iterations"]), show_progress=True,
                                word_name="w" if warm else None, load_initial_params=warm, **kw)
    return A, B, pi, buf.getvalue().splitlines()


@pytest.mark.parametrize("case", golden_cases())
def test_dropin_matches_reference(case, tmp_path, monkeypatch):
    d = load(case)
    A, B, pi, lines = run_dropin(d, tmp_path, monkeypatch)
    assert_params(A, d["out_A"], "A")
    assert_params(B, d["out_B"], "B")
    assert_params(pi, d["out_pi"], "pi")
    assert lines == list(d["stdout"]), "printed progress differs from the reference"


@pytest.mark.parametrize("topology", ["auto", "dense"])
@pytest.mark.parametrize("case", golden_cases())
def test_engine_internals_match_reference(case, topology):
    from hmm_training_amd.engine import BaumWelchEngine
    d = load(case)
    N, M = int(d["N"]), int(d["M"])
    with BaumWelchEngine(N, M, topology=topology) as eng:
        eng.set_observations(observations(d))
        eng.set_params(d["init_pi"], d["init_A"], d["init_B"])
        trace = []
        st = eng.train(float(d["epsilon"]), int(d["max_iterations"]), lambda k, L, df: trace.append((L, df)))
        assert st.iterations == int(d["iterations"])
        assert_ll([t[0] for t in trace], d["trace_L"])
        assert_ll(eng.loglik(), d["trace_logP"][-1])
        pi, A, B = eng.params(normalise=False)
        with np.errstate(under="ignore"):
            assert_params(pi, np.exp(d["trace_log_pi"][-1]), "log_pi")
            assert_params(A, np.exp(d["trace_log_A"][-1]), "log_A")
            assert_params(B, np.exp(d["trace_log_B"][-1]), "log_B")
        # forward-only scorer (hmm_testing.py:49-104) under the returned model
        eng.set_params(d["out_pi"], d["out_A"], d["out_B"])
        assert_ll(eng.score(), d["score_loglik"])


def random_problem(rng, N, K, R, tmax, topology):
    lengths = rng.integers(1, tmax + 1, size=R)
    lengths[0] = tmax
    obs = [rng.integers(0, K, size=int(t)) for t in lengths]
    if topology == "left_to_right":
        A = np.zeros((N, N))
        for i in range(N):
            A[i, i] = rng.uniform(0.3, 0.9)
            if i + 1 < N:
                A[i, i + 1] = 1 - A[i, i]
            else:
                A[i, i] = 1.0
        pi = np.zeros(N)
        pi[0] = 0.8
        pi[1:] = 0.2 / max(N - 1, 1)
        if N == 1:
            pi[0] = 1.0
    else:
        A = rng.dirichlet(np.ones(N), size=N)
        pi = rng.dirichlet(np.ones(N))
    B = rng.dirichlet(np.full(K, 0.5), size=N)
    return obs, pi, A, B


SWEEP = [(N, K, topo) for N in (1, 2, 3, 4, 5, 7, 8, 9, 12, 16) for K, topo in ((16, "dense"), (256, "left_to_right"))]
SWEEP += [(8, 700, "dense"), (8, 700, "left_to_right"), (16, 300, "dense"), (17, 40, "dense"), (24, 128, "dense"),
          (33, 64, "dense"), (40, 96, "dense"), (48, 200, "dense"), (49, 50, "dense"), (64, 300, "dense"),
          (64, 1024, "dense")]


SAFE_SWEEP = [(N, K, topo) for (N, K, topo) in SWEEP if N in (2, 5, 8, 16)]


@pytest.mark.parametrize("N,K,topology,safe", [c + (False,) for c in SWEEP] + [c + (True,) for c in SAFE_SWEEP])
def test_training_vs_oracle_random(N, K, topology, safe, oracle):
    from hmm_training_amd.engine import BaumWelchEngine, to_csr
    rng = np.random.default_rng(1000 * N + K)
    obs, pi, A, B = random_problem(rng, N, K, R=37, tmax=90, topology=topology)
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 1e-6, 3, pi, A, B)
    with BaumWelchEngine(N, K, topology=topology, safe_scaling=safe) as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        assert eng.topology == topology
        trace = []
        eng.train(1e-6, 3, lambda k, L, df: trace.append(L))
        assert_ll(trace, ref.trace_L)
        assert_ll(eng.loglik(), ref.logP)
        p2, A2, B2 = eng.params(normalise=True)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")


@pytest.mark.parametrize("N,equal", [(24, False), (64, False), (64, True)])
@pytest.mark.parametrize("wq", ["1", "0"])
def test_wide_work_queue_vs_oracle(N, equal, wq, oracle, monkeypatch):
    """The wide E-step with more 16-sequence tiles than CUs runs as a work queue of forward and backward
    sweeps (estep_mfma.hpp, WQ; HMMBW_WIDE_WQ=1 forces it above one tile per CU, 0 keeps one tile per
    workgroup): 3 EM iterations against
    the oracle (hmm_training.py:351-514), ragged and equal lengths, both forms."""
    import torch
    from hmm_training_amd.engine import BaumWelchEngine, to_csr
    monkeypatch.setenv("HMMBW_WIDE_WQ", wq)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    R = 16 * ncu + 16 * 21 + 5  # tiles > CUs (the queue form), the last tile partly filled
    K = 64
    rng = np.random.default_rng(31 * N + int(equal))
    obs, pi, A, B = random_problem(rng, N, K, R=R, tmax=24, topology="dense")
    if equal:
        obs = [rng.integers(0, K, size=24) for _ in range(R)]
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 1e-9, 3, pi, A, B)
    with BaumWelchEngine(N, K, topology="dense") as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        assert eng.work_queue_active == (wq == "1")
        trace = []
        eng.train(1e-9, 3, lambda k, L, df: trace.append(L))
        assert_ll(trace, ref.trace_L)
        assert_ll(eng.loglik(), ref.logP)
        p2, A2, B2 = eng.params(normalise=True)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")


def test_wide_work_queue_timeout_is_an_error(oracle):
    """The work queue's bounded wait (estep_mfma.hpp): a backward sweep whose forward has not finished
    within HMMBW_OPT_WQ_TIMEOUT_MS stops EM with HMMBW_E_TIMEOUT, reported by the status calls, instead of
    reading alpha_hat that may not be there.  A 0-ms bound expires before the first look at the flag, so
    the first iteration fails; the next run (reset re-arms the queue) with the default bound then matches
    the oracle (hmm_training.py:351-514)."""
    import torch
    from hmm_training_amd._lib import HMMBW_E_TIMEOUT, HMMBWError
    from hmm_training_amd.engine import BaumWelchEngine, to_csr
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    N, K, R = 32, 64, 16 * ncu + 16 * 9 + 3
    rng = np.random.default_rng(77)
    obs, pi, A, B = random_problem(rng, N, K, R=R, tmax=24, topology="dense")
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 1e-9, 2, pi, A, B)
    with BaumWelchEngine(N, K, topology="dense") as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        eng.set_work_queue(1, timeout_ms=0)
        assert eng.work_queue_active
        eng.reset(1e-9, 2)
        eng.enqueue_iterations(2)
        with pytest.raises(HMMBWError) as ei:
            eng.status()
        assert ei.value.code == HMMBW_E_TIMEOUT
        assert "work-queue" in str(ei.value)
        eng.set_params(pi, A, B)
        eng.set_work_queue(1, timeout_ms=10000)
        trace = []
        eng.train(1e-9, 2, lambda k, L, df: trace.append(L))
        assert_ll(trace, ref.trace_L)
        p2, A2, B2 = eng.params(normalise=True)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")


@pytest.mark.parametrize("topology", ["dense", "left_to_right"])
def test_estep_statistics_vs_oracle(topology, oracle):
    import torch
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout, to_csr
    rng = np.random.default_rng(7)
    N, K = 8, 256
    obs, pi, A, B = random_problem(rng, N, K, R=200, tmax=160, topology=topology)
    off, sym = to_csr(obs)
    s = oracle.estep_logstats(off, sym.astype(np.int64), N, K, pi, A, B)
    with BaumWelchEngine(N, K, topology=topology) as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        eng.reset(1e-6, 10)
        stats = eng.make_stats_buffer()
        from hmm_training_amd._lib import check
        import ctypes
        check(eng._lib.hmmbw_estep(eng._ctx, ctypes.c_void_p(stats.data_ptr())))
        torch.cuda.synchronize()
        got = StatsLayout(N, K).decode(stats.cpu().numpy())
        assert_ll(eng.loglik(), s.logP)
    np.testing.assert_allclose(got["pi_num"], np.exp(s.log_pi_num), rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(got["xi"], np.exp(s.log_xi), rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(got["gamma_den_excl"], np.exp(s.log_gden_excl), rtol=1e-9)
    np.testing.assert_allclose(got["gamma_den_all"], np.exp(s.log_gden_all), rtol=1e-9)
    np.testing.assert_allclose(got["B_num"], np.exp(s.log_bnum), rtol=1e-9, atol=1e-300)
    lp = s.logP[np.isfinite(s.logP)]
    assert np.isclose(StatsLayout.lse_of_pairs(got["ll_pairs"]), oracle.lse(lp), rtol=1e-12)


def test_full_size_cfg3_properties(oracle):
    """BASELINE cfg3 size (R=10,000, T=200, N=8, K=256): size-independent properties of one E-step
    plus oracle parity on a sample of sequences."""
    import ctypes
    import torch
    from hmm_training_amd._lib import check
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(3)
    R, T, N, K = 10_000, 200, 8, 256
    sym = rng.integers(0, K, size=(R, T))
    pi, A, B = default_initial_params(N, K)
    B = rng.dirichlet(np.full(K, 2.0), size=N)
    with BaumWelchEngine(N, K) as eng:
        eng.set_observations(offsets=np.arange(R + 1) * T, symbols=sym.reshape(-1))
        eng.set_params(pi, A, B)
        assert eng.topology == "left_to_right"
        eng.reset(0.0, 1)
        stats = eng.make_stats_buffer()
        check(eng._lib.hmmbw_estep(eng._ctx, ctypes.c_void_p(stats.data_ptr())))
        torch.cuda.synchronize()
        g = StatsLayout(N, K).decode(stats.cpu().numpy())
        ll = eng.loglik()
    assert np.all(np.isfinite(ll))
    np.testing.assert_allclose(g["B_num"].sum(1), g["gamma_den_all"], rtol=1e-11)
    np.testing.assert_allclose(g["xi"].sum(1), g["gamma_den_excl"], rtol=1e-11)
    assert np.isclose(g["pi_num"].sum(), R, rtol=1e-12)
    assert np.isclose(g["gamma_den_all"].sum(), R * T, rtol=1e-12)
    pick = rng.choice(R, size=48, replace=False)
    ref = oracle.forward_loglik(np.arange(len(pick) + 1) * T, sym[pick].reshape(-1).astype(np.int64), N, K, pi, A, B)
    np.testing.assert_allclose(ll[pick], ref, rtol=1e-11)
    assert np.isclose(StatsLayout.lse_of_pairs(g["ll_pairs"]), oracle.lse(ll), rtol=1e-12)


def test_converged_iterations_are_noops():
    from hmm_training_amd.engine import BaumWelchEngine
    d = load("converge")
    N, M = int(d["N"]), int(d["M"])
    with BaumWelchEngine(N, M) as eng:
        eng.set_observations(observations(d))
        eng.set_params(d["init_pi"], d["init_A"], d["init_B"])
        st = eng.train(1e-6, 100)
        assert st.done and st.converged and st.iterations == int(d["iterations"])
        before = eng.params(normalise=False)
        eng.enqueue_iterations(5)
        st2, _ = eng.status()
        assert st2.iterations == st.iterations
        after = eng.params(normalise=False)
    for x, y in zip(before, after):
        np.testing.assert_array_equal(x, y)


def test_error_behaviour():
    from hmm_training_amd.hmm_training import hmm_training
    with pytest.raises(IndexError):
        hmm_training([np.array([1, 2]), np.array([], dtype=np.int64)], N=4, M=8, show_progress=False,
                     load_initial_params=False)
    with pytest.raises(IndexError):
        hmm_training([np.array([1, 9])], N=4, M=8, show_progress=False, load_initial_params=False)
    with pytest.raises(UnboundLocalError):
        hmm_training([np.array([1, 2])], N=4, M=8, max_iterations=0, show_progress=False,
                     load_initial_params=False)


def test_score_matrix_and_timing():
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_classes import HMMTrained
    from hmm_training_amd.hmm_testing import calculate_log_likelihood, score_matrix
    d = load("n8_k256_cfg2")
    obs = observations(d)
    m = HMMTrained(8, 256, d["out_A"], d["out_B"], d["out_pi"], "w")
    S = score_matrix(obs, [m, m])
    assert_ll(S[:, 0], d["score_loglik"])
    assert_ll(S[:, 1], d["score_loglik"])
    assert np.isclose(calculate_log_likelihood(obs[0], m), d["score_loglik"][0], rtol=LL_RTOL)
    with BaumWelchEngine(8, 256) as eng:
        eng.set_observations(obs)
        eng.set_params(d["init_pi"], d["init_A"], d["init_B"])
        eng.timing(1)
        eng.reset(0.0, 4)
        eng.enqueue_iterations(4)
        ms, n = eng.timing(0)
        assert n == 4 and ms > 0


@pytest.mark.parametrize("N,topology", [(8, "left_to_right"), (8, "dense"), (40, "dense")])
@pytest.mark.parametrize("equal_lengths", [True, False])
def test_pathological_emissions_fall_back_to_safe_scaling(N, topology, equal_lengths, oracle):
    """A symbol with probability 1e-200 in every state collapses the lagged scaling; the small kernel
    must detect it and redo the wave with per-step normalisation, and the wide (MFMA) kernel's per-step
    power-of-two normalisation must absorb it, both matching the log-domain oracle."""
    from hmm_training_amd.engine import BaumWelchEngine, to_csr
    rng = np.random.default_rng(99)
    K = 32
    obs, pi, A, B = random_problem(rng, N, K, R=24, tmax=60, topology=topology)
    if equal_lengths:
        obs = [rng.integers(0, K, size=60) for _ in range(24)]
    B[:, 3] = 1e-200
    B /= B.sum(1, keepdims=True)
    for o in obs:
        o[::4] = 3  # frequent, nearly impossible symbol
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 1e-6, 2, pi, A, B)
    assert np.all(np.isfinite(ref.logP))
    with BaumWelchEngine(N, K, topology=topology) as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        trace = []
        eng.train(1e-6, 2, lambda k, L, df: trace.append(L))
        assert_ll(trace, ref.trace_L)
        assert_ll(eng.loglik(), ref.logP)
        p2, A2, B2 = eng.params(normalise=True)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")


@pytest.mark.parametrize("merge,copies", [(True, 4), (False, 1), (False, 4)])
@pytest.mark.parametrize("case", ["n8_k256_cfg2", "n4_k16_default", "converge", "dense_n6"])
def test_engine_variants_match_reference(case, merge, copies):
    """The separate-M-step-kernel and multi-copy accumulation variants give the reference's results."""
    from hmm_training_amd.engine import BaumWelchEngine
    d = load(case)
    N, M = int(d["N"]), int(d["M"])
    with BaumWelchEngine(N, M, merge_mstep=merge, stat_copies=copies) as eng:
        eng.set_observations(observations(d))
        eng.set_params(d["init_pi"], d["init_A"], d["init_B"])
        trace = []
        st = eng.train(float(d["epsilon"]), int(d["max_iterations"]), lambda k, L, df: trace.append(L))
        assert st.iterations == int(d["iterations"])
        assert_ll(trace, d["trace_L"])
        pi, A, B = eng.params(normalise=True)
    assert_params(A, d["out_A"], "A")
    assert_params(B, d["out_B"], "B")
    assert_params(pi, d["out_pi"], "pi")


@pytest.mark.parametrize("case", ["n8_k256_t200", "converge", "zero_prob_seq", "dense_n16", "n64_k1024_tiny"])
@pytest.mark.parametrize("world", [2, 3, 5])
def test_multirank_estep_mstep_in_process(case, world):
    """The multi-rank path (hmmbw_estep -> sum of the packed statistics -> hmmbw_mstep) with `world`
    engines in one process on cuda:0; the all-reduce is a torch sum.  Must match the reference run
    on the unsharded data (hmm_training.py:351-514).  Ranks with an empty shard (more ranks than
    sequences: n64_k1024_tiny holds 2) contribute zero statistics and still run every M-step."""
    import torch
    from hmm_training_amd.engine import BaumWelchEngine, shard_bounds
    d = load(case)
    N, M = int(d["N"]), int(d["M"])
    obs = observations(d)
    bounds = shard_bounds([len(o) for o in obs], world)
    engines, bufs = [], []
    for r, (lo, hi) in enumerate(bounds):
        e = BaumWelchEngine(N, M, rank=r, world_size=world)
        e.set_observations(obs[lo:hi], n_seq_global=len(obs))
        engines.append(e)
    for e in engines:
        e.set_params(d["init_pi"], d["init_A"], d["init_B"])
        e.reset(float(d["epsilon"]), int(d["max_iterations"]))
        bufs.append(e.make_stats_buffer())
    import ctypes
    from hmm_training_amd._lib import check
    for _ in range(int(d["max_iterations"]) + 1):
        for e, b in zip(engines, bufs):
            check(e._lib.hmmbw_estep(e._ctx, ctypes.c_void_p(b.data_ptr())))
        tot = torch.stack(bufs).sum(0)
        for e, b in zip(engines, bufs):
            b.copy_(tot)
            check(e._lib.hmmbw_mstep(e._ctx, ctypes.c_void_p(b.data_ptr()), len(obs)))
    torch.cuda.synchronize()
    for e in engines:
        st, recs = e.status(0, int(d["iterations"]))
        assert st.done and st.iterations == int(d["iterations"])
        assert_ll([L for L, _ in recs], d["trace_L"])
        pi, A, B = e.params(normalise=True)
        assert_params(A, d["out_A"], "A")
        assert_params(B, d["out_B"], "B")
        assert_params(pi, d["out_pi"], "pi")
        e.close()


def _dropin_worker(rank, world, port, case, tmp, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hmm_training_amd.hmm_training import hmm_training
        d = load(case)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            A, B, pi = hmm_training(observations(d), N=int(d["N"]), M=int(d["M"]), epsilon=float(d["epsilon"]),
                                    max_iterations=int(d["max_iterations"]), show_progress=True,
                                    load_initial_params=False)
        q.put((rank, A, B, pi, buf.getvalue().splitlines()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["n4_k256_default", "n4_k16_default"])
def test_dropin_two_processes_gloo(case, tmp_path):
    """hmm_training under an initialised process group (2 ranks on the one GPU, gloo carrying the
    all-reduce of the device statistics buffer): every rank returns the reference's (A, B, pi)."""
    import multiprocessing as mp
    import socket
    d = load(case)
    if bool(d["load_initial"]):
        pytest.skip("warm-start case")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dropin_worker, args=(r, 2, port, case, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, A, B, pi, lines in res:
        assert_params(A, d["out_A"], f"A rank {rank}")
        assert_params(B, d["out_B"], f"B rank {rank}")
        assert_params(pi, d["out_pi"], f"pi rank {rank}")
        if rank == 0:
            assert lines == list(d["stdout"])
        else:
            assert lines == [], "only rank 0 prints the reference's progress lines"


def test_metrics_jsonl_stream(tmp_path):
    """§5 metrics: BaumWelchEngine.train(metrics=...) appends one JSON line per EM iteration with L,
    diff, ms/iter, utt/s/iter, E-step kernel time and the byte-model roofline fraction."""
    import json
    from hmm_training_amd.engine import BaumWelchEngine
    d = load("converge")
    N, M = int(d["N"]), int(d["M"])
    path = tmp_path / "m.jsonl"
    with BaumWelchEngine(N, M) as eng:
        eng.set_observations(observations(d))
        eng.set_params(d["init_pi"], d["init_A"], d["init_B"])
        st = eng.train(float(d["epsilon"]), int(d["max_iterations"]), metrics=str(path))
    rows = [json.loads(l) for l in path.read_text().splitlines()]
    assert [r["iteration"] for r in rows] == list(range(1, st.iterations + 1))
    assert_ll([r["log_likelihood"] for r in rows], d["trace_L"])
    assert rows[0]["diff"] is None and all(r["estep_us"] > 0 and r["utt_per_s_iter"] > 0 for r in rows)
    assert all(0 < r["roofline_frac"] for r in rows)
