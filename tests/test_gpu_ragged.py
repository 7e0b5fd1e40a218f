"""Ragged waves (sequences of different lengths sharing a wave): the chunks every lane is still inside
of run the unmasked loops, the others mask per lane (hmmbw_device.hpp, forward and backward).  The
length patterns put the wave's shortest sequence (T_min) on and around chunk boundaries, so the
switch between masked and unmasked chunks lands on every residue; 3 EM iterations against the oracle
(hmm_training.py:351-514), with the LR (product tables), dense and N=3 kernels, and the scorer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def lengths(tmin, tmax, n, rng):
    """n lengths in [tmin, tmax] with tmin and tmax both present (one wave's worth or more)."""
    t = rng.integers(tmin, tmax + 1, size=n)
    t[0], t[-1] = tmax, tmin
    return t


@pytest.mark.parametrize("tmin", [1, 7, 8, 9, 10, 16, 17, 25, 33, 40, 41])
@pytest.mark.parametrize("N,K,topology", [(8, 256, "left_to_right"), (8, 64, "dense"), (3, 32, "left_to_right")])
def test_ragged_waves_match_oracle(oracle, tmin, N, K, topology):
    from hmm_training_amd.engine import BaumWelchEngine, to_csr
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(1000 + tmin + N)
    G = 1 << (N - 1).bit_length()
    U = 64 // G
    # several waves: one whose lengths span [tmin, tmin + 70], one exactly tmin long, one mixed
    T = np.concatenate([lengths(tmin, tmin + 70, U, rng), np.full(U, tmin), lengths(tmin, tmin + 9, 2 * U + 3, rng)])
    obs = [rng.integers(0, K, size=int(t)) for t in T]
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    B = rng.dirichlet(np.full(K, 2.0), size=N)
    with BaumWelchEngine(N, K, topology=topology) as e:
        e.set_observations(obs)
        e.set_params(pi, A, B)
        score0 = e.score()
        trace = []
        st = e.train(0.0, 3, lambda k, L, d: trace.append(L))
        p2, A2, B2 = e.params(normalise=False)
        ll = e.loglik()
    off, sym = to_csr(obs)
    sym = sym.astype(np.int64)
    np.testing.assert_allclose(score0, oracle.forward_loglik(off, sym, N, K, pi, A, B), rtol=1e-9)
    ref = oracle.hmm_training(off, sym, N, K, 0.0, 3, pi, A, B)
    assert st.iterations == 3
    np.testing.assert_allclose(trace, ref.trace_L, rtol=1e-9)
    with np.errstate(under="ignore"):
        for mine, theirs in ((p2, np.exp(ref.log_pi)), (A2, np.exp(ref.log_A)), (B2, np.exp(ref.log_B))):
            assert np.all(np.abs(mine - theirs) <= 1e-6 * np.abs(theirs) + 1e-15)
    np.testing.assert_allclose(ll, ref.logP, rtol=1e-9)
