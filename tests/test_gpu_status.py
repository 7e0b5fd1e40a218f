"""Non-blocking status snapshots (hmmbw_status_post / hmmbw_status_wait) and the pipelined drop-in
train loop built on them (engine.train; the reference's loop is hmm_training.py:346-514).

A snapshot taken after n queued iterations reports n (separate M-step kernels) or n - 1 (merged
M-step still pending) iterations, and its records are the same numbers a synchronous
hmmbw_get_status returns later; train() reports every iteration exactly once, in order, and stops on
the same iteration as the oracle."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def _engine(N, K, R, seed, merge=True, topology="left_to_right"):
    from hmm_training_amd.engine import BaumWelchEngine
    from hmm_training_amd.hmm_training import default_initial_params
    rng = np.random.default_rng(seed)
    obs = [rng.integers(0, K, size=int(t)) for t in rng.integers(30, 200, size=R)]
    pi, A, B = default_initial_params(N, K)
    e = BaumWelchEngine(N, K, topology=topology, merge_mstep=merge)
    e.set_observations(obs)
    e.set_params(pi, A, B)
    return e, obs, (pi, A, B)


@pytest.mark.parametrize("merge", [True, False])
def test_snapshot_lags_at_most_one_iteration_and_matches_sync_records(merge):
    e, _, _ = _engine(8, 64, 500, 7, merge)
    with e:
        e.reset(0.0, 100)
        e.enqueue_iterations(3)
        t0 = ctypes.c_int64()
        assert e._lib.hmmbw_status_post(e._ctx, 0, ctypes.byref(t0)) == 0
        e.enqueue_iterations(5)  # queued behind the snapshot
        t1 = ctypes.c_int64()
        assert e._lib.hmmbw_status_post(e._ctx, 0, ctypes.byref(t1)) == 0
        st0, recs0 = e._wait_status(t0.value, 0)
        assert st0.iterations == (2 if merge else 3)
        assert not st0.done
        st1, recs1 = e._wait_status(t1.value, 0)
        assert st1.iterations == (7 if merge else 8)
        stf, recsf = e.status(0, 8)  # synchronous (flushes the pending M-step)
        assert stf.iterations == 8
        assert recs1 == recsf[: st1.iterations]
        assert recs0 == recsf[: st0.iterations]
        # a ticket older than the last two is refused
        t2 = ctypes.c_int64()
        assert e._lib.hmmbw_status_post(e._ctx, 0, ctypes.byref(t2)) == 0
        from hmm_training_amd._lib import Status
        s = Status()
        assert e._lib.hmmbw_status_wait(e._ctx, t0.value, ctypes.byref(s), None, 0, 0) != 0


@pytest.mark.parametrize("max_it,eps", [(1, 0.0), (2, 0.0), (37, 0.0), (200, 1e-4)])
def test_pipelined_train_reports_every_iteration_once(oracle, max_it, eps):
    from hmm_training_amd.engine import to_csr
    e, obs, (pi, A, B) = _engine(5, 32, 300, 11)
    seen = []
    with e:
        st = e.train(eps, max_it, lambda k, L, d: seen.append((k, L, d)))
        _, recs = e.status(0, st.iterations)
    assert [k for k, _, _ in seen] == list(range(st.iterations))
    assert [(L, d) for _, L, d in seen] == recs
    off, sym = to_csr(obs)
    ref = oracle.hmm_training(off, sym.astype(np.int64), 5, 32, eps, max_it, pi, A, B)
    assert st.iterations == len(ref.trace_L)
    np.testing.assert_allclose([L for _, L, _ in seen], ref.trace_L, rtol=1e-9)
    assert bool(st.converged) == (st.iterations < max_it)


@pytest.mark.parametrize("merge", [True, False])
def test_live_mirror_matches_sync_records_and_resets(merge):
    """HMMBW_OPT_LIVE_STATUS: the records the M-steps mirror into pinned host memory are the numbers a
    synchronous hmmbw_get_status returns; a wait for more iterations than the queued launches can record
    falls back to the device status once the stream is idle; after a reset the previous run's mirror
    no longer satisfies a wait."""
    e, _, _ = _engine(8, 64, 400, 9, merge)
    with e:
        e.live_status(True)
        e.reset(0.0, 100)
        e.enqueue_iterations(6)
        # merged: launch e + 1 records iteration e, so 6 launches record 5 before the final flush
        want = 5 if merge else 6
        st, recs = e.wait_live(want, 0, want)
        assert st.iterations == want and not st.done
        # nothing will record a 7th iteration: the wait returns the device status when the stream drains
        st2, _ = e.wait_live(want + 3)
        assert st2.iterations == want
        stf, recsf = e.status(0, 6)  # synchronous, flushes the pending M-step
        assert recs == recsf[:want]
        # a new run: the mirror of the old one (6 iterations) must not satisfy a wait for 2
        e.reset(0.0, 100)
        e.enqueue_iterations(3)
        st3, recs3 = e.wait_live(2, 0, 2)
        assert st3.iterations == 2
        st4, recs4 = e.status(0, 3)
        assert recs3 == recs4[:2]
        # stop rule: max_iterations = 4 on a fresh run, more launches than that queued
        e.reset(0.0, 4)
        e.enqueue_iterations(8)
        st5, _ = e.wait_live(100)
        assert st5.done and st5.iterations == 4
        e.live_status(False)
        with pytest.raises(Exception):
            e.wait_live(1)
