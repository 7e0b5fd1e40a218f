"""GPU parity of the grouped launches (hmmbw_group_*): several word models trained by one grouped
E-step launch per EM iteration and scored by one launch, each member against the oracle run alone
(the reference trains word by word, HMM/main.py:147-152, and scores pair by pair,
HMM/hmm_testing.py:139-161).  Same tolerances as test_gpu_parity.py; iteration counts, stop flags
and printed lines exact."""
import contextlib
import io

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


def word_set(n_words, N, K, R=20, seed=0, dense=False, tlo=40, thi=121):
    """cfg2-shaped synthetic words: R sequences each, T ~ U[tlo, thi), skewed symbols, own warm start."""
    rng = np.random.default_rng(seed)
    from hmm_training_amd.hmm_training import default_initial_params
    words = []
    for w in range(n_words):
        pi, A, B = default_initial_params(N, K)
        B = 0.5 * B + 0.5 * rng.dirichlet(np.full(K, 0.5), size=N)
        if dense:
            A = 0.5 * A + 0.5 * rng.dirichlet(np.ones(N), size=N)
        hot = rng.dirichlet(np.full(K, 0.3))
        obs = [rng.choice(K, size=int(t), p=hot) for t in rng.integers(tlo, thi, size=R)]
        words.append((obs, pi, A, B))
    return words


def csr(obs):
    off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
    return off, np.concatenate(obs).astype(np.int64)


def oracle_run(oracle, obs, N, K, eps, maxit, pi, A, B):
    off, sym = csr(obs)
    return oracle.hmm_training(off, sym, N, K, eps, maxit, pi, A, B)


@pytest.mark.parametrize("N,K,dense,maxit,merge", [(8, 256, False, 6, True), (8, 256, True, 4, True),
                                                  (4, 64, False, 100, True), (3, 16, True, 60, True),
                                                  (16, 64, True, 3, True), (8, 256, False, 5, False)])
def test_group_train_matches_each_word_alone(oracle, N, K, dense, maxit, merge):
    """merge=False: every member's M-step is its own kernel between two grouped launches."""
    from hmm_training_amd.engine import BaumWelchEngine, EngineGroup
    words = word_set(10 if N <= 8 else 3, N, K, seed=N * 7 + K, dense=dense)
    engines = []
    for obs, pi, A, B in words:
        e = BaumWelchEngine(N, K, device=0, merge_mstep=merge)
        e.set_observations(obs)
        e.set_params(pi, A, B)
        engines.append(e)
    traces = [[] for _ in words]
    with EngineGroup(engines) as grp:
        sts = grp.train(1e-6, maxit, lambda m, k, L, d: traces[m].append((k, L, d)))
    for m, (obs, pi, A, B) in enumerate(words):
        ref = oracle_run(oracle, obs, N, K, 1e-6, maxit, pi, A, B)
        assert sts[m].iterations == ref.iterations, f"word {m}"
        assert [k for k, _, _ in traces[m]] == list(range(ref.iterations))
        np.testing.assert_allclose([L for _, L, _ in traces[m]], ref.trace_L, rtol=LL_RTOL)
        p2, A2, B2 = engines[m].params(normalise=True)
        assert_params(A2, ref.A, f"A[{m}]")
        assert_params(B2, ref.B, f"B[{m}]")
        assert_params(p2, ref.pi, f"pi[{m}]")
        engines[m].close()


def test_group_members_stop_at_their_own_iteration(oracle):
    """Words converge at different iterations; later iterations are no-ops for the stopped ones."""
    from hmm_training_amd.engine import BaumWelchEngine, EngineGroup
    words = word_set(6, 4, 16, R=4, seed=5, tlo=8, thi=30)
    engines = []
    for obs, pi, A, B in words:
        e = BaumWelchEngine(4, 16, device=0)
        e.set_observations(obs)
        e.set_params(pi, A, B)
        engines.append(e)
    with EngineGroup(engines) as grp:
        sts = grp.train(1e-6, 200)
    its = []
    for m, (obs, pi, A, B) in enumerate(words):
        ref = oracle_run(oracle, obs, 4, 16, 1e-6, 200, pi, A, B)
        its.append(ref.iterations)
        assert sts[m].iterations == ref.iterations and sts[m].converged
        p2, A2, B2 = engines[m].params()
        assert_params(A2, ref.A, f"A[{m}]")
        assert_params(B2, ref.B, f"B[{m}]")
        engines[m].close()
    assert len(set(its)) > 1, "fixture should stop the words at different iterations"


@pytest.mark.parametrize("N,K,dense", [(8, 256, False), (8, 256, True), (5, 32, False), (16, 64, True)])
def test_group_score_matches_oracle(oracle, N, K, dense):
    from hmm_training_amd.engine import BaumWelchEngine, EngineGroup
    words = word_set(7, N, K, R=33, seed=11 + N, dense=dense)
    test_obs = words[0][0] + words[1][0]
    engines = []
    for _, pi, A, B in words:
        e = BaumWelchEngine(N, K, device=0)
        e.set_observations(test_obs)
        e.set_params(pi, A, B)
        engines.append(e)
    with EngineGroup(engines) as grp:
        cols = grp.score()
    off, sym = csr(test_obs)
    for m, (_, pi, A, B) in enumerate(words):
        ref = oracle.forward_loglik(off, sym, N, K, pi, A, B)
        np.testing.assert_allclose(cols[m], ref, rtol=LL_RTOL)
        engines[m].close()


def test_group_rejects_mixed_shapes():
    from hmm_training_amd._lib import HMMBWError
    from hmm_training_amd.engine import BaumWelchEngine, EngineGroup
    (o1, p1, A1, B1), = word_set(1, 4, 16, seed=1)
    (o2, p2, A2, B2), = word_set(1, 5, 16, seed=2)
    e1, e2 = BaumWelchEngine(4, 16, device=0), BaumWelchEngine(5, 16, device=0)
    e1.set_observations(o1), e1.set_params(p1, A1, B1)
    e2.set_observations(o2), e2.set_params(p2, A2, B2)
    with pytest.raises(HMMBWError):
        EngineGroup([e1, e2])
    e1.close(), e2.close()


def test_score_matrix_groups_mixed_models(oracle):
    """score_matrix buckets models by shape: LR and dense words, plus a wide (N=20) one alone."""
    from hmm_training_amd.hmm_classes import HMMTrained
    from hmm_training_amd.hmm_testing import score_matrix
    lr = word_set(3, 8, 64, R=10, seed=21)
    dn = word_set(2, 8, 64, R=10, seed=22, dense=True)
    wd = word_set(1, 20, 64, R=10, seed=23, dense=True)
    models = [HMMTrained(states=len(pi), symbols=64, A=A, B=B, Pi=pi, word=f"w{i}")
              for i, (_, pi, A, B) in enumerate(lr + dn + wd)]
    test_obs = lr[0][0] + dn[0][0]
    S = score_matrix(test_obs, models, device=0)
    off, sym = csr(test_obs)
    for m, h in enumerate(models):
        ref = oracle.forward_loglik(off, sym, h.states, 64, h.Pi, h.A, h.B)
        np.testing.assert_allclose(S[:, m], ref, rtol=LL_RTOL)


def test_hmm_training_group_equals_word_by_word(tmp_path, monkeypatch):
    """Same returned parameters and byte-identical stdout as calling hmm_training per word."""
    from hmm_training_amd.hmm_training import hmm_training, hmm_training_group
    monkeypatch.chdir(tmp_path)
    words = word_set(4, 4, 32, R=6, seed=31)
    sets = [w[0] for w in words]
    names = ["up", "down", "left", "right"]
    out_seq, res_seq = io.StringIO(), []
    with contextlib.redirect_stdout(out_seq):
        for obs, name in zip(sets, names):
            res_seq.append(hmm_training(obs, N=4, M=32, max_iterations=25, word_name=name, device=0))
    out_grp = io.StringIO()
    with contextlib.redirect_stdout(out_grp):
        res_grp = hmm_training_group(sets, N=4, M=32, max_iterations=25, word_names=names, device=0)
    assert out_grp.getvalue() == out_seq.getvalue()
    for (A1, B1, p1), (A2, B2, p2) in zip(res_seq, res_grp):
        assert_params(A2, A1, "A")
        assert_params(B2, B1, "B")
        assert_params(p2, p1, "pi")


def test_main_train_grouped_equals_word_by_word(tmp_path, capsys):
    from test_main_cli import make_data
    from hmm_training_amd.hmm_classes import DataStorageHMM
    from hmm_training_amd.main import train_hmm
    data = str(tmp_path / "Data")
    make_data(data, words=("up", "down"))
    capsys.readouterr()
    a = train_hmm(show_progress=True, max_iterations=7, base_dir=data, model_dir=str(tmp_path / "m1"), grouped=False)
    out_a = capsys.readouterr().out
    b = train_hmm(show_progress=True, max_iterations=7, base_dir=data, model_dir=str(tmp_path / "m2"), grouped=True)
    out_b = capsys.readouterr().out
    assert a is not None and b is not None and out_a == out_b
    for h in a:
        s1 = open(tmp_path / "m1" / f"{h.word}.json").read()
        s2 = open(tmp_path / "m2" / f"{h.word}.json").read()
        assert s1 == s2
