"""The engine's own RCCL communicator (hmmbw_comm_init): multi-rank iterations enqueued by
hmmbw_iterate as estep -> ncclAllReduce -> mstep on the engine's stream.  On one GPU it runs with a
1-rank communicator, which takes exactly that sequence; results must match the oracle like the
single-rank path (hmm_training.py:342-514)."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def rccl_path():
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p.encode() if os.path.exists(p) else None


@pytest.mark.parametrize("topology,maxit,N,K,eps,copies,det", [
    ("left_to_right", 8, 8, 256, 1e-6, None, False),   # fused path: E-step into the all-reduce buffer
    ("dense", 5, 8, 256, 1e-6, None, False),
    ("left_to_right", 40, 5, 64, 1e-3, 1, False),      # converges before maxit (device-side stop rule)
    ("dense", 4, 8, 256, 1e-6, 3, False),
    ("dense", 3, 40, 96, 1e-6, None, False),           # wide path: E-step + gather into the all-reduce buffer
    ("left_to_right", 6, 8, 256, 1e-6, None, True),    # deterministic mode: partials, estep path
    ("dense", 3, 40, 96, 1e-6, None, True),            # deterministic wide path: estep + k_reduce_local
])
def test_native_comm_one_rank_matches_oracle(oracle, topology, maxit, N, K, eps, copies, det):
    from hmm_training_amd._lib import check, lib
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(17)
    R = 600
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(40, 220, size=R)]
    pi, A, B = default_initial_params(N, K)
    if topology == "dense":
        A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
    L = lib()
    with BaumWelchEngine(N, K, device=0, stat_copies=copies, deterministic=det) as e:
        check(L.hmmbw_set_rank(e._ctx, 0, 1))
        e.set_observations(obs)
        e.set_params(pi, A, B)
        uid = ctypes.create_string_buffer(128)
        check(L.hmmbw_comm_unique_id(rccl_path(), uid))
        check(L.hmmbw_comm_init(e._ctx, rccl_path(), uid, 0, 1, R))
        e.timing(1)
        trace = []
        st = e.train(eps, maxit, lambda k, Lk, d: trace.append(Lk))
        p2, A2, B2 = e.params()
        ranks, ar_ms, ar_n = e.comm_info()
        assert ranks == 1 and ar_n >= st.iterations and ar_ms > 0  # chunks past convergence still all-reduce
        copy_len = N + N * N + 2 * N + K * N
        if not det:  # fused (small and wide): the copies + one (max, sum exp) pair per rank, 256-B aligned;
            # the wide path all-reduces ONE copy (its B numerator is written once, by the gather)
            nc = 1 if N > 16 else (copies or 2)
            assert e.comm_payload_bytes() == 8 * (-(-(nc * copy_len + 2) // 32) * 32)
        else:
            assert e.comm_payload_bytes() == 8 * e.stats_len
    off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
    ref = oracle.hmm_training(off, np.concatenate(obs).astype(np.int64), N, K, eps, maxit, pi, A, B)
    assert st.iterations == ref.iterations
    np.testing.assert_allclose(trace, ref.trace_L, rtol=1e-9)
    for mine, theirs in ((A2, ref.A), (B2, ref.B), (p2, ref.pi)):
        assert np.all(np.abs(mine - theirs) <= 1e-6 * np.abs(theirs) + 1e-15)


def test_comm_init_rejects_bad_rank():
    from hmm_training_amd._lib import lib
    from hmm_training_amd.engine import BaumWelchEngine
    L = lib()
    with BaumWelchEngine(4, 16, device=0) as e:
        uid = ctypes.create_string_buffer(128)
        assert L.hmmbw_comm_unique_id(rccl_path(), uid) == 0
        assert L.hmmbw_comm_init(e._ctx, rccl_path(), uid, 1, 2, 10) != 0  # set_rank was not called
        assert L.hmmbw_comm_init(e._ctx, rccl_path(), uid, 3, 2, 10) != 0
