"""Full-size BASELINE configurations on the GPU, compared with the oracle on the SAME inputs.

Each case runs the production path (hmmbw_iterate: E-step launches with the merged M-step) for several
EM iterations and checks against oracle.hmm_training (hmm_training.py:351-514, run with OpenMP over
utterances on the host's cores: the same log-domain terms as the serial restatement, merged per thread):
  * every recorded L (:503) at rtol 1e-9, every sequence's log P of the last E-step at rtol 1e-9;
  * the returned (pi, A, B) (:524-541) and the working parameters (exp of the reference's log_pi /
    log_a / log_b) at the north-star tolerance |x - ref| <= 1e-6 |ref| + 1e-15;
then one statistics pass (hmmbw_estep) with the final parameters against oracle.estep_logstats:
  * the COMPLETE packed statistics (pi_num, xi, gamma_den_excl, gamma_den_all, B_num) at rtol 1e-9,
    every log P at rtol 1e-9 and the rank's (max, sum exp) pair against the oracle's LSE;
  * the M-step the kernels apply to them (hmmbw_mstep) against the reference's formulas (:415-497),
    and the sum rules (sum_k B_num = gamma_den_all, sum_j xi = gamma_den_excl, sum pi_num = R,
    sum gamma_den_all = R T).
Configurations: cfg3 (10,000 x 200, N=8, K=256) left-to-right and dense, the cfg4 per-GPU shard
(12,500 x 200) on skewed 'H' symbols, cfg4 whole (100,000 x 200) on one GPU (two iterations), a
full-shape cfg5 slice (512 x 400, N=64, K=1024, dense), the cfg5 per-GPU shard (6,250 x 400), and the
whole cfg5 set (50,000 x 400) on one GPU as four ranks through the split ABI: each quarter's complete
statistics against the oracle on that quarter, and the iteration (L, M-step) against the merged oracle
quarters.
"""
import ctypes
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PARAM_RTOL, PARAM_ATOL, LL_RTOL, STAT_RTOL = 1e-6, 1e-15, 1e-9, 1e-9


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def _symbols(R, T, N, K, kind, seed):
    sys.path.insert(0, ROOT)
    import bench
    return bench.synthetic_symbols(R, T, N, K, kind, seed)


def _params(N, K, topology, seed):
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(seed)
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    B = rng.dirichlet(np.full(K, 2.0), size=N)  # away from uniform so the first M-step moves things
    return pi, A, B


def assert_params(mine, ref, what):
    mine, ref = np.asarray(mine), np.asarray(ref)
    err = np.abs(mine - ref) - (PARAM_RTOL * np.abs(ref) + PARAM_ATOL)
    assert np.all(err <= 0), f"{what}: worst excess {err.max():.3e} at {np.unravel_index(np.argmax(err), err.shape)}"


def host_mstep(g, R):
    """The reference's M-step (hmm_training.py:415-497) in the linear domain, from packed statistics."""
    pi = np.where(g["pi_num"] > 0, g["pi_num"] / R, 0.0)
    den = g["gamma_den_excl"][:, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        A = np.where((den > 0) & (g["xi"] > 0), g["xi"] / den, 0.0)
        gall = g["gamma_den_all"][:, None]
        B = np.where(gall > 0, np.where(g["B_num"] > 0, g["B_num"] / gall, 1e-20), 0.0)
    return pi, A, B


def assert_stats(g, s, R, T):
    """Packed device statistics vs the oracle's log-domain ones (exp), plus the sum rules."""
    with np.errstate(under="ignore"):
        for key, lkey in (("pi_num", "log_pi_num"), ("xi", "log_xi"), ("gamma_den_excl", "log_gden_excl"),
                          ("gamma_den_all", "log_gden_all"), ("B_num", "log_bnum")):
            ref = np.exp(getattr(s, lkey))
            np.testing.assert_allclose(g[key], ref, rtol=STAT_RTOL, atol=1e-300, err_msg=key)
    np.testing.assert_allclose(g["B_num"].sum(1), g["gamma_den_all"], rtol=1e-11)
    np.testing.assert_allclose(g["xi"].sum(1), g["gamma_den_excl"], rtol=1e-11)
    assert np.isclose(g["pi_num"].sum(), R, rtol=1e-12)
    assert np.isclose(g["gamma_den_all"].sum(), R * T, rtol=1e-12)


def statistics_pass(eng, N, K, R):
    """One hmmbw_estep with the current parameters; returns (decoded stats, log P, M-step params)."""
    import torch
    from hmm_training_amd._lib import check
    from hmm_training_amd.engine import StatsLayout
    eng.reset(0.0, 1)
    stats = eng.make_stats_buffer()
    check(eng._lib.hmmbw_estep(eng._ctx, ctypes.c_void_p(stats.data_ptr())))
    torch.cuda.synchronize()
    g = StatsLayout(N, K).decode(stats.cpu().numpy())
    ll = eng.loglik()
    check(eng._lib.hmmbw_mstep(eng._ctx, ctypes.c_void_p(stats.data_ptr()), R))
    return g, ll, eng.params(normalise=False)


def run_vs_oracle(oracle, R, T, N, K, topology, iters, seed, symbols="U", deterministic=False, work_queue=None):
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout
    sym = _symbols(R, T, N, K, symbols, seed)
    off = np.arange(R + 1, dtype=np.int64) * T
    sym64 = sym.astype(np.int64)
    pi, A, B = _params(N, K, topology, seed)
    ref = oracle.hmm_training(off, sym64, N, K, 0.0, iters, pi, A, B)
    assert ref.iterations == iters
    with BaumWelchEngine(N, K, topology=topology, deterministic=deterministic) as eng:
        eng.set_observations(offsets=off, symbols=sym)
        eng.set_params(pi, A, B)
        assert eng.topology == topology
        if work_queue is not None:  # which wide E-step form the library chose on its own (no option set)
            assert eng.work_queue_active == work_queue
        # -------- production iterations, enqueued together (merged M-steps) --------
        eng.reset(0.0, iters)
        eng.enqueue_iterations(iters)
        st, recs = eng.status(0, iters)
        assert st.iterations == iters and st.done and not st.converged
        np.testing.assert_allclose([L for L, _ in recs], ref.trace_L, rtol=LL_RTOL)
        np.testing.assert_allclose(eng.loglik(), ref.logP, rtol=LL_RTOL)  # E-step of the last iteration
        p_out, A_out, B_out = eng.params(normalise=True)
        assert_params(A_out, ref.A, "A")
        assert_params(B_out, ref.B, "B")
        assert_params(p_out, ref.pi, "pi")
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        with np.errstate(under="ignore"):
            assert_params(p_cur, np.exp(ref.log_pi), "log_pi")
            assert_params(A_cur, np.exp(ref.log_A), "log_A")
            assert_params(B_cur, np.exp(ref.log_B), "log_B")
        # -------- statistics pass with the final parameters --------
        g, ll, (p_m, A_m, B_m) = statistics_pass(eng, N, K, R)
    s = oracle.estep_logstats(off, sym64, N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll, s.logP, rtol=LL_RTOL)
    assert_stats(g, s, R, T)
    assert np.isclose(StatsLayout.lse_of_pairs(g["ll_pairs"]), oracle.lse(s.logP), rtol=1e-12)
    hp, hA, hB = host_mstep(g, R)
    np.testing.assert_allclose(p_m, hp, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(A_m, hA, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(B_m, hB, rtol=1e-12, atol=1e-300)


def test_cfg3_full_size_vs_oracle(oracle_mt):
    """BASELINE cfg3: 10,000 x T=200, N=8, K=256, left-to-right (the headline kernel), 4 EM iterations."""
    run_vs_oracle(oracle_mt, 10_000, 200, 8, 256, "left_to_right", 4, seed=3)


def test_cfg3_full_size_dense_vs_oracle(oracle_mt):
    run_vs_oracle(oracle_mt, 10_000, 200, 8, 256, "dense", 3, seed=33)


def test_cfg4_shard_full_size_vs_oracle(oracle_mt):
    """BASELINE cfg4's per-GPU shard: 12,500 x T=200, N=8, K=256, 3 EM iterations, skewed symbols
    (hot symbols contend in the B-numerator histogram)."""
    run_vs_oracle(oracle_mt, 12_500, 200, 8, 256, "left_to_right", 3, seed=4, symbols="H")


def test_cfg4_whole_on_one_gpu_vs_oracle(oracle_mt):
    """BASELINE cfg4 unsharded: 100,000 x T=200, N=8, K=256 on one GPU, two EM iterations + statistics."""
    run_vs_oracle(oracle_mt, 100_000, 200, 8, 256, "left_to_right", 2, seed=44)


def test_cfg5_full_shape_slice_vs_oracle(oracle_mt):
    """BASELINE cfg5's shape (T=400, N=64, K=1024, dense: the fp64-MFMA wide path, k_estep_mfma +
    k_bnum_gather + k_mstep_grid) on 512 sequences, 2 EM iterations, everything against the oracle."""
    run_vs_oracle(oracle_mt, 512, 400, 64, 1024, "dense", 2, seed=55)


def test_cfg5_shard_full_size_vs_oracle(oracle_mt):
    """BASELINE cfg5's per-GPU shard: 6,250 x T=400, N=64, K=1024, dense, 2 EM iterations vs the oracle."""
    run_vs_oracle(oracle_mt, 6_250, 400, 64, 1024, "dense", 2, seed=5)


def test_wide_work_queue_one_context_full_size_vs_oracle(oracle_mt):
    """The wide work queue (a workgroup per forward and per backward sweep, estep_mfma.hpp WQ) as the
    library selects it on its own: ONE context above the 4-tiles-per-CU threshold (18,000 x T=200 = 1,125
    tiles, N=64, K=256, dense), 2 EM iterations and a statistics pass against the oracle
    (hmm_training.py:351-514), including the counter and flag re-arm by the last of 2,250 workgroups."""
    import torch
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    R = 18_000
    assert (R + 15) // 16 > 4 * ncu, "the case must sit above the work queue's threshold"
    run_vs_oracle(oracle_mt, R, 200, 64, 256, "dense", 2, seed=18, work_queue=True)


def test_cfg5_shard_is_not_on_the_work_queue(oracle_mt):
    """The cfg5 per-GPU shard (391 tiles, 1.5 per CU) keeps one workgroup per tile: the queue measured
    slower there (profiles/r4/wide_work_queue_ab.txt)."""
    from hmm_training_amd.engine import BaumWelchEngine
    with BaumWelchEngine(64, 1024, topology="dense") as eng:
        eng.set_observations(offsets=np.arange(6_251, dtype=np.int64) * 400,
                             symbols=np.zeros(6_250 * 400, dtype=np.int32))
        assert not eng.work_queue_active


def test_cfg3_full_size_deterministic_vs_oracle(oracle_mt):
    """cfg3 in deterministic-reduction mode (gamma rows + k_bnum_gather, per-workgroup partials +
    k_det_reduce: no floating-point atomics), 3 EM iterations against the oracle."""
    run_vs_oracle(oracle_mt, 10_000, 200, 8, 256, "left_to_right", 3, seed=31, deterministic=True)


def test_cfg5_slice_deterministic_vs_oracle(oracle_mt):
    """The wide path's deterministic mode (k_estep_mfma<.., DET>: every statistic in its owning lane,
    per-tile partials) at cfg5's shape, 1,024 x 400, N=64, K=1024, 2 EM iterations against the oracle."""
    run_vs_oracle(oracle_mt, 1024, 400, 64, 1024, "dense", 2, seed=56, deterministic=True)


CFG5_WHOLE = dict(R=50_000, T=400, N=64, K=1024, world=4, seed=5)
_cfg5_oracle_parts = {}


@pytest.fixture(scope="module")
def cfg5_whole_gpu():
    """BASELINE cfg5 unsharded: 50,000 x T=400, N=64, K=1024, dense, ONE EM iteration on ONE GPU as four
    ranks of 12,500 sequences (the reference's per-utterance xi allocation, hmm_training.py:328-339, cannot
    run it at all), through the split-iteration ABI, which runs the kernels of a 4-GPU job: each rank's
    partial statistics (the buffer it would all-reduce) and log P are kept for the per-quarter oracle
    comparisons, then the buffers are summed and every rank applies the M-step (:415-514)."""
    import torch
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout, shard_bounds
    c = CFG5_WHOLE
    R, T, N, K, W = c["R"], c["T"], c["N"], c["K"], c["world"]
    sym = _symbols(R, T, N, K, "U", c["seed"])
    pi, A, B = _params(N, K, "dense", c["seed"])
    bounds = shard_bounds([T] * R, W)
    layout = StatsLayout(N, K, W)
    engines, parts = [], []
    try:
        for r, (lo, hi) in enumerate(bounds):
            e = BaumWelchEngine(N, K, rank=r, world_size=W, topology="dense")
            e.set_observations(offsets=np.arange(hi - lo + 1, dtype=np.int64) * T, symbols=sym[lo * T:hi * T],
                               n_seq_global=R)
            e.set_params(pi, A, B)
            e.reset(0.0, 1)
            engines.append(e)
        bufs = [e.iterate_begin() for e in engines]
        torch.cuda.synchronize()
        tot = None
        for (ptr, n), e in zip(bufs, engines):
            x = torch.empty(n, dtype=torch.float64, device="cuda:0")
            torch.cuda.synchronize()
            hip_copy(x.data_ptr(), ptr, 8 * n)
            parts.append(layout.decode(x[:layout.length].cpu().numpy()))
            tot = x.clone() if tot is None else tot + x
        for ptr, n in bufs:
            hip_copy(ptr, tot.data_ptr(), 8 * n)
        logp = [e.loglik() for e in engines]
        for e in engines:
            e.iterate_end()
        res = []
        for e in engines:
            st, recs = e.status(0, 1)
            res.append((st, recs, e.params(normalise=False), e.params(normalise=True)))
    finally:
        for e in engines:
            e.close()
    return dict(sym=sym, params=(pi, A, B), bounds=bounds, parts=parts, logp=logp, res=res, layout=layout)


def hip_copy(dst, src, nbytes):
    import os

    import torch
    h = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    h.hipMemcpy.restype = ctypes.c_int
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    torch.cuda.synchronize()
    assert h.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3) == 0
    torch.cuda.synchronize()


def _cfg5_oracle_part(oracle, run, q):
    if q not in _cfg5_oracle_parts:
        c = CFG5_WHOLE
        lo, hi = run["bounds"][q]
        T, N, K = c["T"], c["N"], c["K"]
        pi, A, B = run["params"]
        _cfg5_oracle_parts[q] = oracle.estep_logstats(np.arange(hi - lo + 1, dtype=np.int64) * T,
                                                      run["sym"][lo * T:hi * T].astype(np.int64), N, K, pi, A, B)
    return _cfg5_oracle_parts[q]


@pytest.mark.parametrize("q", [0, 1, 2, 3])
def test_cfg5_whole_quarter_statistics_vs_oracle(oracle_mt, cfg5_whole_gpu, q):
    """One quarter (12,500 sequences) of the whole cfg5 set: that rank's COMPLETE partial statistics
    (pi_num, xi, gamma_den_excl, gamma_den_all, B_num: hmm_training.py:388-497) at rtol 1e-9, every log P
    (:375-377) at rtol 1e-9 and the rank's (max, sum exp) pair against the oracle on the same sequences."""
    from hmm_training_amd.engine import StatsLayout
    run = cfg5_whole_gpu
    c = CFG5_WHOLE
    lo, hi = run["bounds"][q]
    s = _cfg5_oracle_part(oracle_mt, run, q)
    g = run["parts"][q]
    np.testing.assert_allclose(run["logp"][q], s.logP, rtol=LL_RTOL)
    with np.errstate(under="ignore"):
        for key, lkey in (("pi_num", "log_pi_num"), ("xi", "log_xi"), ("gamma_den_excl", "log_gden_excl"),
                          ("gamma_den_all", "log_gden_all"), ("B_num", "log_bnum")):
            np.testing.assert_allclose(g[key], np.exp(getattr(s, lkey)), rtol=STAT_RTOL, atol=1e-300, err_msg=key)
    assert np.isclose(g["pi_num"].sum(), hi - lo, rtol=1e-12)
    assert np.isclose(g["gamma_den_all"].sum(), (hi - lo) * c["T"], rtol=1e-12)
    pair = g["ll_pairs"][q]
    assert np.all(np.delete(g["ll_pairs"], q, axis=0) == 0.0)  # only this rank's slot is written
    assert np.isclose(StatsLayout.lse_of_pairs(pair), oracle_mt.lse(s.logP), rtol=1e-12)


def test_cfg5_whole_iteration_vs_oracle(oracle_mt, cfg5_whole_gpu):
    """The whole cfg5 set's EM iteration: the oracle's statistics of the four quarters merged (log-sum-exp,
    hmm_training.py:66-79) and its M-step (:415-500), against every rank's parameters after the
    all-reduce (working and returned, :524-541), and L (:503) over all 50,000 log P."""
    run = cfg5_whole_gpu
    c = CFG5_WHOLE
    R, N, K = c["R"], c["N"], c["K"]
    s = oracle_mt.merge_logstats([_cfg5_oracle_part(oracle_mt, run, q) for q in range(c["world"])])
    lpi, la, lb = oracle_mt.mstep_log(R, N, K, s)
    L = oracle_mt.lse(s.logP)
    with np.errstate(under="ignore"):
        epi, eA, eB = np.exp(lpi), np.exp(la), np.exp(lb)
    for r, (st, recs, (p_cur, A_cur, B_cur), (p_out, A_out, B_out)) in enumerate(run["res"]):
        assert st.iterations == 1 and st.done
        assert np.isclose(recs[0][0], L, rtol=LL_RTOL), f"rank {r}"
        assert_params(p_cur, epi, f"log_pi rank {r}")
        assert_params(A_cur, eA, f"log_A rank {r}")
        assert_params(B_cur, eB, f"log_B rank {r}")
        assert_params(p_out, epi / epi.sum(), f"pi rank {r}")
        assert_params(A_out, eA / eA.sum(1, keepdims=True), f"A rank {r}")
        assert_params(B_out, eB / eB.sum(1, keepdims=True), f"B rank {r}")
        for x, y in zip((p_cur, A_cur, B_cur), run["res"][0][2]):
            np.testing.assert_array_equal(x, y)  # replicated: bitwise-identical on every rank


@pytest.mark.parametrize("xact,topology,join", [(None, "left_to_right", None), ("1", "left_to_right", None),
                                                ("3", "left_to_right", None), ("4", "left_to_right", None),
                                                (None, "left_to_right", "0"), ("1", "left_to_right", "0"),
                                                (None, "dense", None), (None, "dense", "0")])
def test_spread_extra_waves_ragged_vs_oracle(oracle_mt, monkeypatch, xact, topology, join):
    """More waves than SIMDs (9,000 ragged sequences = 1,125 waves on 1,024 SIMDs): one full workgroup
    per CU, then workgroups of xact active waves (default 2; HMMBW_XACT forces 1, 3 or 4 = no spread map),
    with inactive waves in them; by default on the joined map (the extra workgroups' waves as waves 4.. of the
    full ones, k_estep_join; dense too since round 6), HMMBW_JOIN=0 the separate workgroups; every statistic and
    the trained model against the oracle (hmm_training.py:351-514)."""
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout, to_csr
    if xact is not None:
        monkeypatch.setenv("HMMBW_XACT", xact)
    if join is not None:
        monkeypatch.setenv("HMMBW_JOIN", join)
    rng = np.random.default_rng(9)
    R, N, K, iters = 9000, 8, 256, 3
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(60, 160, size=R)]
    off, sym = to_csr(obs)
    pi, A, B = _params(N, K, topology, 9)
    ref = oracle_mt.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    with BaumWelchEngine(N, K, topology=topology) as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        lm = eng.launch_map()
        spread = xact != "4"
        assert (lm["workgroups"] > lm["full_workgroups"]) == spread, lm
        assert lm["joined"] == (spread and join != "0"), lm  # round 6: the dense E-step joins too
        eng.reset(0.0, iters)
        eng.enqueue_iterations(iters)
        st, recs = eng.status(0, iters)
        np.testing.assert_allclose([L for L, _ in recs], ref.trace_L, rtol=LL_RTOL)
        np.testing.assert_allclose(eng.loglik(), ref.logP, rtol=LL_RTOL)
        p_out, A_out, B_out = eng.params(normalise=True)
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        g, ll, _ = statistics_pass(eng, N, K, R)
    assert_params(A_out, ref.A, "A")
    assert_params(B_out, ref.B, "B")
    assert_params(p_out, ref.pi, "pi")
    s = oracle_mt.estep_logstats(off, sym.astype(np.int64), N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll, s.logP, rtol=LL_RTOL)
    with np.errstate(under="ignore"):
        for key, lkey in (("pi_num", "log_pi_num"), ("xi", "log_xi"), ("gamma_den_excl", "log_gden_excl"),
                          ("gamma_den_all", "log_gden_all"), ("B_num", "log_bnum")):
            np.testing.assert_allclose(g[key], np.exp(getattr(s, lkey)), rtol=STAT_RTOL, atol=1e-300, err_msg=key)
    assert np.isclose(StatsLayout.lse_of_pairs(g["ll_pairs"]), oracle_mt.lse(s.logP), rtol=1e-12)


@pytest.mark.parametrize("R,join", [(8192, None), (3001, None), (8192, "0")])
def test_joined_map_without_extra_groups_vs_oracle(oracle_mt, monkeypatch, R, join):
    """Round 6: with at most 4 sequence groups per CU (no spread map) the left-to-right E-step still runs the joined
    kernel, one 8-wave workgroup per CU whose waves 4-7 hold no group and only share the table build and the flush
    (HMMBW_JOIN=0: the plain 4-wave workgroups).  R = 8,192 (every SIMD one group) and 3,001 ragged (a partial last
    workgroup); 2 EM iterations and every statistic against the oracle (hmm_training.py:351-514)."""
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout, to_csr
    if join is not None:
        monkeypatch.setenv("HMMBW_JOIN", join)
    rng = np.random.default_rng(R)
    N, K, iters = 8, 256, 2
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(40, 120, size=R)]
    off, sym = to_csr(obs)
    pi, A, B = _params(N, K, "left_to_right", 17)
    ref = oracle_mt.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    with BaumWelchEngine(N, K, topology="left_to_right") as eng:
        eng.set_observations(obs)
        eng.set_params(pi, A, B)
        lm = eng.launch_map()
        assert lm["workgroups"] == lm["full_workgroups"] and not lm["split_extra"], lm
        assert lm["joined"] == (join != "0"), lm
        eng.reset(0.0, iters)
        eng.enqueue_iterations(iters)
        st, recs = eng.status(0, iters)
        np.testing.assert_allclose([L for L, _ in recs], ref.trace_L, rtol=LL_RTOL)
        np.testing.assert_allclose(eng.loglik(), ref.logP, rtol=LL_RTOL)
        p_out, A_out, B_out = eng.params(normalise=True)
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        g, ll, _ = statistics_pass(eng, N, K, R)
    assert_params(A_out, ref.A, "A")
    assert_params(B_out, ref.B, "B")
    assert_params(p_out, ref.pi, "pi")
    s = oracle_mt.estep_logstats(off, sym.astype(np.int64), N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll, s.logP, rtol=LL_RTOL)
    with np.errstate(under="ignore"):
        for key, lkey in (("pi_num", "log_pi_num"), ("xi", "log_xi"), ("gamma_den_excl", "log_gden_excl"),
                          ("gamma_den_all", "log_gden_all"), ("B_num", "log_bnum")):
            np.testing.assert_allclose(g[key], np.exp(getattr(s, lkey)), rtol=STAT_RTOL, atol=1e-300, err_msg=key)
    assert np.isclose(StatsLayout.lse_of_pairs(g["ll_pairs"]), oracle_mt.lse(s.logP), rtol=1e-12)


@pytest.mark.parametrize("join", ["1", "0"])
@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("T,topology,safe", [(203, "left_to_right", False), (203, "dense", False), (9, "left_to_right", False),
                                             (64, "left_to_right", True), (96, "dense", True), (9, "dense", False)])
def test_split_extra_waves_vs_oracle(oracle_mt, monkeypatch, split, T, topology, safe, join):
    """Split extra waves (HMMBW_SPLIT_EXTRA, estep_small_body "split"): 10,000 equal-length sequences put a
    second wave on 226 SIMDs; with the split each such group's backward is cut at chunk nch / 2 and its idle
    partner wave runs the lower half from its own beta pre-sweep, rescaled into the forward's scaling.
    Odd T (a partial top chunk), the two-chunk minimum (T = 9), per-step (safe) scaling, both topologies:
    2 EM iterations and every statistic against the oracle (hmm_training.py:351-514).  join: the joined spread map
    (one 8-wave workgroup per CU, round 6 for the dense kernel: the split groups hand over by an LDS flag) or
    the separate extra workgroups (HMMBW_JOIN_DENSE=0 / HMMBW_JOIN=0)."""
    from hmm_training_amd.engine import BaumWelchEngine
    monkeypatch.setenv("HMMBW_SPLIT_EXTRA", split)
    monkeypatch.setenv("HMMBW_JOIN_DENSE" if topology == "dense" else "HMMBW_JOIN", join)
    R, N, K, iters = 10_000, 8, 256, 2
    sym = _symbols(R, T, N, K, "U", 71 + T)
    off = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = _params(N, K, topology, 71)
    ref = oracle_mt.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    with BaumWelchEngine(N, K, topology=topology, safe_scaling=safe) as eng:
        eng.set_observations(offsets=off, symbols=sym)
        eng.set_params(pi, A, B)
        lm = eng.launch_map()
        assert bool(lm["joined"]) == (join == "1"), lm
        # left-to-right splits on the joined map only (round 6)
        assert bool(lm["split_extra"]) == (split == "1" and (topology == "dense" or join == "1")), lm
        eng.reset(0.0, iters)
        eng.enqueue_iterations(iters)
        st, recs = eng.status(0, iters)
        np.testing.assert_allclose([L for L, _ in recs], ref.trace_L, rtol=LL_RTOL)
        np.testing.assert_allclose(eng.loglik(), ref.logP, rtol=LL_RTOL)
        p_out, A_out, B_out = eng.params(normalise=True)
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        g, ll, _ = statistics_pass(eng, N, K, R)
    assert_params(A_out, ref.A, "A")
    assert_params(B_out, ref.B, "B")
    assert_params(p_out, ref.pi, "pi")
    s = oracle_mt.estep_logstats(off, sym.astype(np.int64), N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll, s.logP, rtol=LL_RTOL)
    assert_stats(g, s, R, T)


@pytest.mark.parametrize("topology", ["dense", "left_to_right"])
@pytest.mark.parametrize("N,R", [(4, 20_000), (5, 10_000), (12, 5_000), (16, 5_000)])
def test_split_extra_waves_other_group_sizes_vs_oracle(oracle_mt, monkeypatch, N, R, topology):
    """The split extra waves at the other lane-group sizes (G = 4, 8 with padding states, 16), dense and
    left-to-right (the joined map): R chosen so that the sequence groups overflow the 1,024 SIMDs by ~22 %
    (the spread map's extra workgroups), T = 72 (9 chunks, an odd count), 2 EM iterations and every statistic
    against the oracle (hmm_training.py:351-514)."""
    from hmm_training_amd.engine import BaumWelchEngine
    monkeypatch.setenv("HMMBW_SPLIT_EXTRA", "1")
    T, K, iters = 72, 64, 2
    sym = _symbols(R, T, N, K, "U", 90 + N)
    off = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = _params(N, K, topology, 90 + N)
    ref = oracle_mt.hmm_training(off, sym.astype(np.int64), N, K, 0.0, iters, pi, A, B)
    with BaumWelchEngine(N, K, topology=topology) as eng:
        eng.set_observations(offsets=off, symbols=sym)
        eng.set_params(pi, A, B)
        lm = eng.launch_map()
        assert lm["extra_waves"] in (1, 2) and lm["workgroups"] > lm["full_workgroups"], lm
        assert lm["split_extra"], lm
        eng.reset(0.0, iters)
        eng.enqueue_iterations(iters)
        st, recs = eng.status(0, iters)
        np.testing.assert_allclose([L for L, _ in recs], ref.trace_L, rtol=LL_RTOL)
        p_out, A_out, B_out = eng.params(normalise=True)
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        g, ll, _ = statistics_pass(eng, N, K, R)
    assert_params(A_out, ref.A, "A")
    assert_params(B_out, ref.B, "B")
    assert_params(p_out, ref.pi, "pi")
    s = oracle_mt.estep_logstats(off, sym.astype(np.int64), N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll, s.logP, rtol=LL_RTOL)
    assert_stats(g, s, R, T)
