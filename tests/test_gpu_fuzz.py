"""Seeded random sweep of the HIP engine against the oracle (hmm_training.py:265-541 restated in
oracle/bw_oracle.c): N in 1..64, M in 1..1024, ragged lengths 1..400, left-to-right and dense
transition matrices, warm starts with zero entries in pi / B, merged and separate M-steps, one or
more statistics copies, lagged and forced per-step scaling.  Every case runs a few EM iterations and
compares the iteration count, every iteration's L, the returned (A, B, pi) and the forward-only scores.
Tolerances as test_gpu_parity.py, plus an absolute 1e-12 on per-sequence log P: with M = 1 symbol every
log P is log(1) = 0 up to rounding (~1e-15), where a relative tolerance means nothing."""
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


def case(i):
    rng = np.random.default_rng(1000 + i)
    N = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 9, 12, 16, 17, 24, 33, 48, 64]))
    M = int(rng.choice([1, 2, 7, 16, 64, 200, 256, 1024]))
    R = int(rng.integers(1, 90))
    T = rng.integers(1, 401, size=R) if rng.random() < 0.7 else np.full(R, int(rng.integers(1, 401)))
    obs = [rng.integers(0, M, size=int(t)) for t in T]
    dense = N > 16 or rng.random() < 0.5
    pi = rng.dirichlet(np.ones(N))
    if dense:
        A = rng.dirichlet(np.ones(N), size=N)
        if N > 2 and rng.random() < 0.3:  # some exact zeros in a dense matrix
            A[rng.integers(0, N, size=N), rng.integers(0, N, size=N)] = 0.0
            A[:, 0] += 1e-3
            A /= A.sum(1, keepdims=True)
    else:
        A = np.zeros((N, N))
        for j in range(N):
            if j + 1 < N:
                A[j, j] = rng.uniform(0.2, 0.95)
                A[j, j + 1] = 1.0 - A[j, j]
            else:
                A[j, j] = 1.0
    B = rng.dirichlet(np.full(M, 0.7), size=N)
    if rng.random() < 0.3:  # zero-probability entries in the warm start
        B[rng.integers(0, N), rng.integers(0, M)] = 0.0
        pi[rng.integers(0, N)] = 0.0
        if pi.sum() == 0:
            pi[0] = 1.0
    opts = dict(merge=bool(rng.random() < 0.7), copies=int(rng.choice([1, 2, 3])), safe=bool(rng.random() < 0.2))
    return N, M, obs, pi, A, B, dense, opts


@pytest.mark.parametrize("i", range(40))
def test_fuzz_against_oracle(oracle, i):
    from hmm_training_amd.engine import BaumWelchEngine
    N, M, obs, pi, A, B, dense, opts = case(i)
    maxit = 3
    off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
    sym = np.concatenate(obs).astype(np.int64)
    ref = oracle.hmm_training(off, sym, N, M, 1e-6, maxit, pi, A, B)
    with BaumWelchEngine(N, M, device=0, topology="dense" if dense else "auto", merge_mstep=opts["merge"],
                         stat_copies=opts["copies"], safe_scaling=opts["safe"]) as e:
        e.set_observations(obs)
        e.set_params(pi, A, B)
        sc = e.score()
        trace = []
        st = e.train(1e-6, maxit, lambda k, L, d: trace.append(L))
        p2, A2, B2 = e.params()
    assert st.iterations == ref.iterations
    np.testing.assert_allclose(trace, ref.trace_L, rtol=LL_RTOL)
    assert_params(A2, ref.A, "A")
    assert_params(B2, ref.B, "B")
    assert_params(p2, ref.pi, "pi")
    scr = oracle.forward_loglik(off, sym, N, M, pi, A, B)
    assert np.array_equal(np.isneginf(sc), np.isneginf(scr))
    f = np.isfinite(scr)
    np.testing.assert_allclose(sc[f], scr[f], rtol=LL_RTOL, atol=1e-12)
