"""GPU parity of the left-to-right kernel with two states per lane (estep_lr2.hpp, 5 <= N <= 8):
EM runs and the forward-only scorer against the oracle (hmm_training.py:342-514,
hmm_testing.py:49-104) and against the one-state-per-lane kernel (HMMBW_OPT_LR_PAIRS = 0), on ragged
lengths, T = 1, sequence counts that leave the last 16-sequence tile partly empty, and the
per-step-scaling fall back.  Same tolerances as test_gpu_parity.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAM_RTOL, PARAM_ATOL, LL_RTOL = 1e-6, 1e-15, 1e-9


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def assert_params(mine, ref, what):
    mine, ref = np.asarray(mine), np.asarray(ref)
    err = np.abs(mine - ref) - (PARAM_RTOL * np.abs(ref) + PARAM_ATOL)
    assert np.all(err <= 0), f"{what}: worst excess {err.max():.3e}"


def problem(N, K, R, lengths, seed, tiny_b=False):
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(seed)
    pi, A, B = default_initial_params(N, K)
    idx = np.arange(N - 1)
    A[idx, idx] = rng.uniform(0.3, 0.9, size=N - 1)
    A[idx, idx + 1] = 1.0 - A[idx, idx]
    B = 0.5 * B + 0.5 * rng.dirichlet(np.full(K, 0.5), size=N)
    if tiny_b:  # magnitudes that leave [2^-900, 2^900] within a few hundred steps: per-step fall back
        B = B * 1e-30
    if lengths == "equal":
        T = np.full(R, int(rng.integers(1, 300)))
    elif lengths == "short":
        T = rng.integers(1, 4, size=R)
    else:
        T = rng.integers(1, 260, size=R)
    obs = [rng.integers(0, K, size=int(t)) for t in T]
    return obs, pi, A, B


def run(obs, N, K, pi, A, B, maxit, pairs, merge=True, safe=False):
    from hmm_training_amd._lib import OPT_LR_PAIRS, check
    from hmm_training_amd.engine import BaumWelchEngine
    with BaumWelchEngine(N, K, device=0, topology="left_to_right", merge_mstep=merge, safe_scaling=safe) as e:
        check(e._lib.hmmbw_set_option(e._ctx, OPT_LR_PAIRS, 1 if pairs else 0))
        e.set_observations(obs)
        e.set_params(pi, A, B)
        sc = e.score()
        trace = []
        st = e.train(1e-6, maxit, lambda k, L, d: trace.append(L))
        p2, A2, B2 = e.params()
        ll = e.loglik()
    return st, trace, (p2, A2, B2), sc, ll


@pytest.mark.parametrize("N", [5, 6, 7, 8])
@pytest.mark.parametrize("R,lengths", [(29, "ragged"), (17, "equal"), (40, "short"), (333, "ragged"), (64, "equal")])
def test_lr2_matches_oracle_and_one_state_kernel(oracle, N, R, lengths):
    K = 64
    obs, pi, A, B = problem(N, K, R, lengths, seed=N * 1000 + R)
    off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
    sym = np.concatenate(obs).astype(np.int64)
    ref = oracle.hmm_training(off, sym, N, K, 1e-6, 4, pi, A, B)
    st, trace, (p2, A2, B2), sc, ll = run(obs, N, K, pi, A, B, 4, True)
    assert st.iterations == ref.iterations
    np.testing.assert_allclose(trace, ref.trace_L, rtol=LL_RTOL)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")
    np.testing.assert_allclose(sc, oracle.forward_loglik(off, sym, N, K, pi, A, B), rtol=LL_RTOL)
    st_v, trace_v, (p3, A3, B3), sc_v, ll_v = run(obs, N, K, pi, A, B, 4, False)
    np.testing.assert_allclose(trace, trace_v, rtol=1e-12)
    np.testing.assert_allclose(ll, ll_v, rtol=1e-12)


@pytest.mark.parametrize("safe", [False, True])
def test_lr2_scaling_fallback(oracle, safe):
    """Emissions ~1e-32 push the lagged scaling out of range: the wave must redo its forward with
    per-step normalisation (or is forced to with HMMBW_OPT_SAFE_SCALING) and still match."""
    N, K, R = 8, 32, 70
    obs, pi, A, B = problem(N, K, R, "ragged", seed=77, tiny_b=True)
    off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
    sym = np.concatenate(obs).astype(np.int64)
    ref = oracle.hmm_training(off, sym, N, K, 1e-6, 3, pi, A, B)
    st, trace, (p2, A2, B2), sc, ll = run(obs, N, K, pi, A, B, 3, True, safe=safe)
    np.testing.assert_allclose(trace, ref.trace_L, rtol=LL_RTOL)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")


@pytest.mark.parametrize("merge", [True, False])
def test_lr2_cfg3_shape(oracle, merge):
    """cfg3 shape: 10,000 sequences x T = 200, N = 8, K = 256, left-to-right: both kernels agree and a
    sample of sequences' log P matches the oracle."""
    N, K, R = 8, 256, 10000
    obs, pi, A, B = problem(N, K, R, "equal", seed=5)
    obs = [o[:1] if i % 997 == 0 else o for i, o in enumerate(obs)]  # a few T = 1 sequences
    st, trace, (p2, A2, B2), sc, ll = run(obs, N, K, pi, A, B, 3, True, merge)
    st_v, trace_v, (p3, A3, B3), sc_v, ll_v = run(obs, N, K, pi, A, B, 3, False, merge)
    np.testing.assert_allclose(trace, trace_v, rtol=1e-12)
    assert_params(A2, A3, "A")
    assert_params(B2, B3, "B")
    pick = np.arange(0, R, 409)
    sub = [obs[i] for i in pick]
    off = np.concatenate([[0], np.cumsum([len(o) for o in sub])]).astype(np.int64)
    np.testing.assert_allclose(sc[pick], oracle.forward_loglik(off, np.concatenate(sub).astype(np.int64), N, K,
                                                                pi, A, B), rtol=LL_RTOL)
