"""Deterministic-reduction mode (HMMBW_OPT_DETERMINISTIC, SURVEY §5 "bitwise-stable CI"): no
floating-point atomics, so two runs on the same input give bitwise-identical parameters, iteration
records and per-sequence log-likelihoods; and the results still match the oracle (hmm_training.py
:351-514) to the parity tolerance.  The default mode sums with fp64 atomics (order not fixed)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def problem(N, K, R, topology, seed):
    rng = np.random.default_rng(seed)
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(20, 260, size=R)]
    from hmm_training_amd.hmm_training import default_initial_params
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    B = rng.dirichlet(np.full(K, 2.0), size=N)
    return obs, pi, A, B


def run(obs, pi, A, B, N, K, iters, det, merge=True):
    from hmm_training_amd.engine import BaumWelchEngine
    with BaumWelchEngine(N, K, deterministic=det, merge_mstep=merge) as e:
        e.set_observations(obs)
        e.set_params(pi, A, B)
        trace = []
        e.train(0.0, iters, lambda k, L, d: trace.append((L, d)))
        p, a, b = e.params(normalise=False)
        return np.array(trace), p, a, b, e.loglik()


@pytest.mark.parametrize("N,K,topology,R", [(8, 256, "left_to_right", 3000), (8, 256, "dense", 3000),
                                            (5, 64, "dense", 3000), (3, 32, "left_to_right", 3000),
                                            (13, 100, "dense", 3000),
                                            # wide path (fp64 MFMA, k_estep_mfma<NT, false, true>)
                                            (40, 64, "dense", 150), (64, 1024, "dense", 120),
                                            (20, 50, "left_to_right", 150)])
def test_deterministic_runs_are_bitwise_equal_and_match_oracle(oracle, N, K, topology, R):
    from hmm_training_amd.engine import to_csr
    obs, pi, A, B = problem(N, K, R, topology, 41 + N)
    r1 = run(obs, pi, A, B, N, K, 4, True)
    r2 = run(obs, pi, A, B, N, K, 4, True)
    for x, y in zip(r1, r2):
        assert np.array_equal(x, y), "deterministic mode differs between runs"
    r3 = run(obs, pi, A, B, N, K, 4, True, merge=False)  # separate M-step kernel: same statistics
    for x, y in zip(r1, r3):
        np.testing.assert_allclose(x, y, rtol=1e-13, atol=1e-300)
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), N, K, 0.0, 4, pi, A, B)
    np.testing.assert_allclose(r1[0][:, 0], ref.trace_L, rtol=1e-9)
    with np.errstate(under="ignore"):
        for mine, theirs in ((r1[1], np.exp(ref.log_pi)), (r1[2], np.exp(ref.log_A)), (r1[3], np.exp(ref.log_B))):
            assert np.all(np.abs(mine - theirs) <= 1e-6 * np.abs(theirs) + 1e-15)
    np.testing.assert_allclose(r1[4], ref.logP, rtol=1e-9)


def test_deterministic_option_rules():
    from hmm_training_amd._lib import OPT_DETERMINISTIC, HMMBWError, lib
    from hmm_training_amd.engine import BaumWelchEngine
    with pytest.raises(HMMBWError):
        BaumWelchEngine(16, 4096, deterministic=True)  # emission tables too large for LDS: unsupported
    with BaumWelchEngine(8, 256) as e:
        e.set_observations([np.array([1, 2, 3])])
        assert lib().hmmbw_set_option(e._ctx, OPT_DETERMINISTIC, 1) != 0  # after the observations
