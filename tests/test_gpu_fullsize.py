"""Full-size BASELINE configurations on the GPU (cfg3, cfg4 shard and whole, cfg5 shard), several EM
iterations each, through the production path (hmmbw_iterate: E-step with the merged M-step).

At these sizes the oracle cannot replay whole runs in seconds, so parity rests on size-independent
properties, all from hmm_training.py:351-514:
  * EM monotonicity: sum_r log P_r never decreases from one iteration to the next (Baum-Welch is an
    EM algorithm for the product of the sequence likelihoods; the reference's convergence scalar
    L = LSE_r log P_r is recorded too and must be finite);
  * E-step sum rules on a fresh statistics pass with the final parameters:
    sum_k B_num[j, k] = gamma_den_all[j], sum_j xi[i, j] = gamma_den_excl[i],
    sum_i pi_num[i] = number of sequences with finite log P, sum_j gamma_den_all[j] = sum_r T_r;
  * the M-step the kernels apply to those statistics equals the reference's formulas evaluated on
    the host from the same statistics (:415-497, incl. the 1e-20 floor), to 1e-12;
  * returned (A, B, pi) rows sum to 1 (:524-541);
  * 48 sampled sequences' log P against oracle.forward_loglik (hmm_testing.py:49-104 = the E-step's
    alpha recursion) at rtol 1e-9, and the per-workgroup LSE pairs against the oracle's LSE.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


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


def host_mstep(g, R):
    """The reference's M-step (hmm_training.py:415-497) in the linear domain, from packed statistics."""
    pi = np.where(g["pi_num"] > 0, g["pi_num"] / R, 0.0)
    den = g["gamma_den_excl"][:, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        A = np.where((den > 0) & (g["xi"] > 0), g["xi"] / den, 0.0)
        gall = g["gamma_den_all"][:, None]
        B = np.where(gall > 0, np.where(g["B_num"] > 0, g["B_num"] / gall, 1e-20), 0.0)
    return pi, A, B


def run_fullsize(oracle, R, T, N, K, topology, iters, seed, symbols="U"):
    import torch
    from hmm_training_amd._lib import check
    from hmm_training_amd.engine import BaumWelchEngine, StatsLayout
    sym = _symbols(R, T, N, K, symbols, seed)
    off = np.arange(R + 1, dtype=np.int64) * T
    pi, A, B = _params(N, K, topology, seed)
    with BaumWelchEngine(N, K, topology=topology) as eng:
        eng.set_observations(offsets=off, symbols=sym)
        eng.set_params(pi, A, B)
        assert eng.topology == topology
        # -------- several production iterations (hmmbw_iterate), one at a time --------
        eng.reset(0.0, iters)
        sums = []
        for k in range(iters):
            eng.enqueue_iterations(1)
            st, recs = eng.status(k, 1)
            assert st.iterations == k + 1
            lp = eng.loglik()  # log P_r under the parameters that entered iteration k
            assert np.all(np.isfinite(lp)), f"iteration {k}: non-finite log P"
            assert np.isfinite(recs[0][0])
            assert np.isclose(recs[0][0], oracle.lse(lp), rtol=1e-12)  # L = LSE_r log P_r (:503)
            sums.append(float(np.sum(lp)))
        assert st.done and not st.converged
        for a, b in zip(sums, sums[1:]):
            assert b >= a - 1e-9 * abs(a), f"EM decreased sum log P: {a} -> {b}"
        p_out, A_out, B_out = eng.params(normalise=True)
        for m in (A_out, B_out):
            np.testing.assert_allclose(m.sum(1), 1.0, rtol=1e-12)
        assert np.isclose(p_out.sum(), 1.0, rtol=1e-12)
        p_cur, A_cur, B_cur = eng.params(normalise=False)
        # -------- a statistics pass with the current parameters: sum rules + M-step --------
        eng.reset(0.0, 1)
        stats = eng.make_stats_buffer()
        check(eng._lib.hmmbw_estep(eng._ctx, ctypes.c_void_p(stats.data_ptr())))
        torch.cuda.synchronize()
        g = StatsLayout(N, K).decode(stats.cpu().numpy())
        ll = eng.loglik()
        check(eng._lib.hmmbw_mstep(eng._ctx, ctypes.c_void_p(stats.data_ptr()), R))
        p_m, A_m, B_m = eng.params(normalise=False)
    assert np.all(np.isfinite(ll))
    np.testing.assert_allclose(g["B_num"].sum(1), g["gamma_den_all"], rtol=1e-11)
    np.testing.assert_allclose(g["xi"].sum(1), g["gamma_den_excl"], rtol=1e-11)
    assert np.isclose(g["pi_num"].sum(), R, rtol=1e-12)
    assert np.isclose(g["gamma_den_all"].sum(), R * T, rtol=1e-12)
    assert np.isclose(g["gamma_den_excl"].sum(), R * (T - 1), rtol=1e-12)
    hp, hA, hB = host_mstep(g, R)
    np.testing.assert_allclose(p_m, hp, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(A_m, hA, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(B_m, hB, rtol=1e-12, atol=1e-300)
    rng = np.random.default_rng(seed + 1)
    pick = np.sort(rng.choice(R, size=48, replace=False))
    ref = oracle.forward_loglik(np.arange(len(pick) + 1) * T, sym.reshape(R, T)[pick].reshape(-1).astype(np.int64),
                                N, K, p_cur, A_cur, B_cur)
    np.testing.assert_allclose(ll[pick], ref, rtol=1e-9)
    from hmm_training_amd.engine import StatsLayout as SL
    assert np.isclose(SL.lse_of_pairs(g["ll_pairs"]), oracle.lse(ll), rtol=1e-12)
    return sums


def test_cfg3_full_size_multi_iteration(oracle):
    """BASELINE cfg3: 10,000 x T=200, N=8, K=256, left-to-right, 4 EM iterations."""
    run_fullsize(oracle, 10_000, 200, 8, 256, "left_to_right", 4, seed=3)


def test_cfg3_full_size_dense(oracle):
    run_fullsize(oracle, 10_000, 200, 8, 256, "dense", 3, seed=33)


def test_cfg4_shard_full_size(oracle):
    """BASELINE cfg4's per-GPU shard: 12,500 x T=200, N=8, K=256, 3 EM iterations, skewed symbols
    (hot symbols contend in the B-numerator histogram)."""
    run_fullsize(oracle, 12_500, 200, 8, 256, "left_to_right", 3, seed=4, symbols="H")


def test_cfg4_whole_on_one_gpu(oracle):
    """BASELINE cfg4 unsharded: 100,000 x T=200, N=8, K=256 on one GPU (fits HBM), 3 EM iterations."""
    run_fullsize(oracle, 100_000, 200, 8, 256, "left_to_right", 3, seed=44)


def test_cfg5_shard_full_size(oracle):
    """BASELINE cfg5's per-GPU shard: 6,250 x T=400, N=64, K=1024, dense A (the fp64-MFMA wide path,
    k_estep_mfma + k_bnum_gather + k_mstep_grid), 2 EM iterations."""
    run_fullsize(oracle, 6_250, 400, 64, 1024, "dense", 2, seed=5)
