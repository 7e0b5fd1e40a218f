"""The oracle (oracle/bw_oracle.c, a C restatement of hmm_training.py:265-541) against the golden
vectors produced by running the reference itself (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from conftest import GOLDEN, golden_cases


def load(case):
    return np.load(f"{GOLDEN}/bw_{case}.npz", allow_pickle=False)


def same_inf_pattern(a, b):
    return np.array_equal(np.isneginf(a), np.isneginf(b)) and np.array_equal(np.isposinf(a), np.isposinf(b))


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_matches_reference(case, oracle):
    d = load(case)
    N, M = int(d["N"]), int(d["M"])
    r = oracle.hmm_training(d["offsets"], d["symbols"], N, M, float(d["epsilon"]), int(d["max_iterations"]),
                            d["init_pi"], d["init_A"], d["init_B"])
    assert r.iterations == int(d["iterations"])
    # per-iteration convergence scalar (hmm_training.py:503)
    np.testing.assert_allclose(r.trace_L, d["trace_L"], rtol=1e-12, atol=0)
    # per-sequence log P of the last iteration (:377)
    lp = d["trace_logP"][-1]
    assert same_inf_pattern(r.logP, lp)
    fin = np.isfinite(lp)
    np.testing.assert_allclose(r.logP[fin], lp[fin], rtol=1e-12)
    # unnormalised log parameters after the last M-step: same -inf pattern, abs error in log space
    for mine, ref in ((r.log_pi, d["trace_log_pi"][-1]), (r.log_A, d["trace_log_A"][-1]),
                      (r.log_B, d["trace_log_B"][-1])):
        assert same_inf_pattern(mine, ref)
        f = np.isfinite(ref)
        np.testing.assert_allclose(mine[f], ref[f], rtol=0, atol=1e-10)
    # returned (A, B, pi), :524-541
    for mine, key in ((r.A, "out_A"), (r.B, "out_B"), (r.pi, "out_pi")):
        np.testing.assert_allclose(mine, d[key], rtol=1e-10, atol=1e-15)


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_forward_score(case, oracle):
    d = load(case)
    N, M = int(d["N"]), int(d["M"])
    sc = oracle.forward_loglik(d["offsets"], d["symbols"], N, M, d["out_pi"], d["out_A"], d["out_B"])
    ref = d["score_loglik"]
    assert same_inf_pattern(sc, ref)
    f = np.isfinite(ref)
    np.testing.assert_allclose(sc[f], ref[f], rtol=1e-12)


def test_oracle_vq(oracle):
    d = np.load(f"{GOLDEN}/vq_k64.npz", allow_pickle=False)
    assert np.array_equal(oracle.vq(d["frames"], d["centroids"]), d["symbols"])


def test_oracle_estep_stats_consistency(oracle):
    """Sum rules of the E-step statistics: sum_j xi(i,j) = gamma_den_excl(i); sum_k B_num = gamma_den_all."""
    d = load("dense_n6")
    N, M = int(d["N"]), int(d["M"])
    s = oracle.estep_logstats(d["offsets"], d["symbols"], N, M, d["init_pi"], d["init_A"], d["init_B"])
    np.testing.assert_allclose(np.exp(s.log_xi).sum(1), np.exp(s.log_gden_excl), rtol=1e-12)
    np.testing.assert_allclose(np.exp(s.log_bnum).sum(1), np.exp(s.log_gden_all), rtol=1e-12)
    np.testing.assert_allclose(np.exp(s.log_pi_num).sum(), len(d["offsets"]) - 1, rtol=1e-12)
