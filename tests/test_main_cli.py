"""The main.py train/test counterpart (hmm_training_amd/main.py) on a synthetic Data/ tree laid out
like the reference's (HMM/main.py:46-197; frame/codebook JSON as CodeVector/codevector_classes.py)."""
import json
import os

import numpy as np
import pytest


def make_data(root, words=("up", "down"), n_train=4, n_test=2, K=16, seed=0):
    """Codebook of K centroids in two clusters; word w's frames are drawn near its cluster."""
    rng = np.random.default_rng(seed)
    cent = rng.normal(size=(K, 13))
    cent[: K // 2, 1:] += 4.0
    cent[K // 2:, 1:] -= 4.0
    os.makedirs(os.path.join(root, "CodeVector"), exist_ok=True)
    with open(os.path.join(root, "CodeVector", "codevector.json"), "w") as fh:
        json.dump([{"mfcc": c.tolist(), "id": i} for i, c in enumerate(cent)], fh, indent=2)
    for purpose, n in (("TrainHMM", n_train), ("Test", n_test)):
        for w, word in enumerate(words):
            for r in range(n):
                d = os.path.join(root, purpose, word, f"{word}-{r:02d}")
                os.makedirs(d, exist_ok=True)
                T = int(rng.integers(20, 40))
                base = cent[rng.integers(0, K // 2, size=T) + (K // 2) * w]
                frames = base + 0.1 * rng.normal(size=base.shape)
                with open(os.path.join(d, f"{word}-{r:02d}_frames.json"), "w") as fh:
                    json.dump([{"mfcc_vector": f.tolist(), "frame_number": t} for t, f in enumerate(frames)], fh)
    return cent


def test_loaders(tmp_path):
    from hmm_training_amd.main import load_all_recordings_by_word, load_mfcc_centroids
    make_data(str(tmp_path))
    cents = load_mfcc_centroids(str(tmp_path), print_messages=False)
    assert len(cents) == 16 and cents[3].id == 3 and cents[0].mfcc.shape == (13,)
    recs = load_all_recordings_by_word(str(tmp_path), "TrainHMM", print_messages=False, print_summary=False)
    assert sorted(recs) == ["down", "up"] and all(len(v) == 4 for v in recs.values())
    assert all(20 <= len(r) < 40 for v in recs.values() for r in v)
    assert load_all_recordings_by_word(str(tmp_path), "Nope", print_messages=False) == {}


@pytest.mark.gpu
def test_train_then_test_matches_oracle(tmp_path, oracle):
    from hmm_training_amd.hmm_classes import DataStorageHMM
    from hmm_training_amd.hmm_training import default_initial_params, get_observations
    from hmm_training_amd.main import load_all_recordings_by_word, load_mfcc_centroids, test, train_hmm
    data, models = str(tmp_path / "Data"), str(tmp_path / "models")
    make_data(data)
    trained = train_hmm(show_progress=False, max_iterations=5, base_dir=data, model_dir=models)
    assert trained is not None and sorted(h.word for h in trained) == ["down", "up"]
    cents = load_mfcc_centroids(data, print_messages=False)
    recs = load_all_recordings_by_word(data, "TrainHMM", print_messages=False, print_summary=False)
    pi0, A0, B0 = default_initial_params(4, len(cents))
    for word, rec in recs.items():
        obs = get_observations(rec, cents)
        off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int64)
        ref = oracle.hmm_training(off, np.concatenate(obs).astype(np.int64), 4, len(cents), 1e-6, 5, pi0, A0, B0)
        saved = DataStorageHMM.load_hmm(word, models, print_messages=False)
        np.testing.assert_allclose(saved.A, ref.A, rtol=1e-6, atol=1e-15)
        np.testing.assert_allclose(saved.B, ref.B, rtol=1e-6, atol=1e-15)
        np.testing.assert_allclose(saved.Pi, ref.pi, rtol=1e-6, atol=1e-15)
    true_labels, predicted = test(base_dir=data, model_dir=models)
    assert len(true_labels) == 4 and true_labels == predicted
