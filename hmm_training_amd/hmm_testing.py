"""Forward-only scoring, the drop-in for HMM/hmm_testing.py (calculate_log_likelihood :49-104,
test_hmm :107-163), on the MI355X engine.

``score_matrix`` is the batched form: every (sequence, model) log-likelihood in one grouped HIP launch,
instead of the reference's per-pair Python forward pass.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .engine import BaumWelchEngine, EngineGroup
from .hmm_classes import HMMTrained
from .hmm_training import get_observations


def score_matrix(observations: Sequence[np.ndarray], models: Sequence[HMMTrained], device=None) -> np.ndarray:
    """[len(observations), len(models)] log P(O_r | model_m) (hmm_testing.py:49-104 per entry).

    Models of one shape (N, M, resolved topology) are scored together by ONE grouped launch over all
    (sequence, model) pairs (hmmbw_group_score); a model the grouped kernel does not take (N > 16,
    tables too large for LDS) gets its own launch."""
    out = np.full((len(observations), len(models)), -np.inf)
    if len(observations) == 0 or len(models) == 0:
        return out
    engines = []
    try:
        for hmm in models:
            N, M = int(hmm.states), int(np.asarray(hmm.B).shape[1])
            eng = BaumWelchEngine(N, M, device=device)
            engines.append(eng)
            eng.set_observations(observations)
            eng.set_params(np.asarray(hmm.Pi), np.asarray(hmm.A), np.asarray(hmm.B))
        buckets = {}
        for m, eng in enumerate(engines):
            key = (eng.N, eng.M, eng.topology) if eng.N <= 16 else ("single", m)
            buckets.setdefault(key, []).append(m)
        for members in buckets.values():
            try:
                grp = EngineGroup([engines[m] for m in members])
            except Exception:
                grp = None
            if grp is None:
                for m in members:
                    out[:, m] = engines[m].score()
                continue
            with grp:
                for m, col in zip(members, grp.score()):
                    out[:, m] = col
    finally:
        for eng in engines:
            eng.close()
    return out


def calculate_log_likelihood(recording_observations: np.ndarray, hmm: HMMTrained) -> float:
    """log P(O | lambda) of one sequence under one linear-domain model (hmm_testing.py:49-104)."""
    return float(score_matrix([np.asarray(recording_observations)], [hmm])[0, 0])


def test_hmm(all_hmm: List[HMMTrained], test_recordings_dict: Dict[str, list], base_dir="../Data",
             show_progress=False, centroids=None) -> Tuple[List[str], List[str]]:
    """Classify every test recording by the max forward log-likelihood (hmm_testing.py:107-163)."""
    print("Starting HMM testing...")
    if centroids is None:
        from .io import load_centroids
        centroids = load_centroids(os.path.join(base_dir, "CodeVector", "codevector.json"))
    print("Phase 1: Converting recordings to observations...")
    observations: Dict[str, List[np.ndarray]] = {}
    for word, recordings in test_recordings_dict.items():
        print(f"  Converting {len(recordings)} recordings for word: '{word}'")
        observations[word] = get_observations(recordings, centroids)
    print("Phase 2: Testing all recording-HMM combinations...")
    true_labels, predicted = [], []
    for true_word, obs_list in observations.items():
        print(f"Testing {len(obs_list)} recordings for word: '{true_word}'")
        scores = score_matrix(obs_list, all_hmm) if obs_list else np.zeros((0, len(all_hmm)))
        for r in range(len(obs_list)):
            best, pred = -float("inf"), None
            for m, hmm in enumerate(all_hmm):
                if scores[r, m] > best:  # strict '>' keeps the first best model (:151)
                    best, pred = scores[r, m], hmm.word
            if show_progress:
                print(f"  Recording {r + 1} likelihoods: {dict(zip([h.word for h in all_hmm], scores[r]))}")
                print(f"  True: '{true_word}' -> Predicted: '{pred}'")
            true_labels.append(true_word)
            predicted.append(pred if pred else "unknown")
    return true_labels, predicted
