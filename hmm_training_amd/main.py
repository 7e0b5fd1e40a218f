"""``train`` / ``test`` entry points of the reference's HMM/main.py (:46-197) on the MI355X engine.

    python -m hmm_training_amd.main train [--max-iterations 2] [--data ../Data]
    python -m hmm_training_amd.main test  [--data ../Data]

Same on-disk layout as the reference:
* ``<data>/CodeVector/codevector.json`` — the codebook;
* ``<data>/<TrainHMM|Test>/<word>/<recording>/*_frames.json`` — the recordings;
* ``<data>/ResultsHMM/<word>.json`` — the trained models (DataStorageHMM's default directory).

The same messages are printed, in the same order. Two things differ:
* training runs every word model together, one grouped E-step launch per EM iteration
  (``hmm_training_group``; each model still stops on its own rule, so the saved models equal the
  reference's word-by-word training); ``grouped=False`` trains word by word through the drop-in
  ``training_with_save``;
* testing goes through ``test_hmm`` (one scoring launch for all (recording, model) pairs).
The confusion-matrix plot (``create_confusion_matrix``, matplotlib) is out of scope; ``test``
returns the labels instead.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import logging
import sys
import os
import random
from collections import defaultdict
from pathlib import Path
from typing import Dict, List, Optional

from .hmm_classes import DataStorageHMM, HMMTrained
from .hmm_testing import test_hmm
from .hmm_training import get_observations, hmm_training_group, training_with_save
from .io import Centroid, Frame, load_centroids, load_frames

logger = logging.getLogger(__name__)


def load_all_recordings_by_word(base_dir="../Data", purpose="TrainHMM", print_messages=True,
                                print_summary=True) -> Dict[str, List[List[Frame]]]:
    """{word: [recording frames, ...]} from ``<base_dir>/<purpose>/<word>/<rec>/*_frames.json``
    (main.py:46-102; the first frame file of each recording directory, directory order)."""
    all_words: Dict[str, List[List[Frame]]] = defaultdict(list)
    purpose_path = Path(base_dir) / purpose
    if not purpose_path.exists():
        print(f"Warning: Directory {purpose_path} does not exist")
        return dict(all_words)
    if print_messages:
        print(f"Loading recordings from {purpose_path}")
    for word_dir in purpose_path.iterdir():
        if not word_dir.is_dir():
            continue
        if print_messages:
            print(f"  Processing word: {word_dir.name}")
        for recording_dir in word_dir.iterdir():
            if not recording_dir.is_dir():
                continue
            frame_files = list(recording_dir.glob("*_frames.json"))
            if frame_files:
                frames = load_frames(str(frame_files[0]))
                if print_messages:
                    print(f"  Loaded {len(frames)} frames from {frame_files[0]}")
                if frames:
                    all_words[word_dir.name].append(frames)
                    if print_messages:
                        print(f"    Added recording with {len(frames)} frames from {recording_dir.name}")
    result = dict(all_words)
    if print_summary:
        print("\nSummary:")
        print(f"  Total words: {len(result)}")
        for word, recordings in result.items():
            print(f"    {word}: {len(recordings)} recordings with {sum(len(r) for r in recordings)} total frames")
    return result


def load_mfcc_centroids(base_dir="../Data", print_messages=True) -> List[Centroid]:
    """The codebook ``<base_dir>/CodeVector/codevector.json`` (main.py:105-130), [] if absent."""
    path = os.path.join(base_dir, "CodeVector", "codevector.json")
    if not os.path.exists(path):
        return []
    centroids = load_centroids(path)
    if print_messages:
        print("\nLoading codevector:")
        print(f"  Loaded codevector with {len(centroids)} centroids")
        c = random.choice(centroids)
        print("  Example random centroid:")
        print(f"   id: {c.id}")
        print(f"   Power: {c.mfcc[0]:.3f}")
        print(" ".join(f"   {x:.3f}" for x in c.mfcc[1:]))
        print("\n")
    return centroids


def _train_grouped(recordings_by_word, centroids, show_progress, max_iterations, load_initial_params,
                   model_dir, n_states=4) -> Optional[List[HMMTrained]]:
    """All words in one group (hmm_training_group), printing each word's lines in word order exactly
    as the word-by-word loop does.  None when the grouped run cannot start (the caller then runs the
    word-by-word loop, which reproduces the reference's partial output and error for bad input)."""
    heads, obs_sets, words = [], [], []
    try:
        for word_name, word_recordings in recordings_by_word.items():
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                print(f"\nTraining HMM for word: '{word_name}' with {len(word_recordings)} recordings")
                print("Converting recordings to observations...")  # training_with_save, hmm_training.py:215-247
                observations = get_observations(word_recordings, centroids)
                print(f"Generated {len(observations)} observation sequences")
                print(f"Sequence lengths: {[len(obs) for obs in observations]}")
                print("Starting Baum-Welch training...")
            heads.append(buf.getvalue())
            obs_sets.append(observations)
            words.append(word_name)
        parts: List[str] = []
        results = hmm_training_group(obs_sets, N=n_states, M=len(centroids), max_iterations=max_iterations,
                                     show_progress=show_progress, word_names=words,
                                     load_initial_params=load_initial_params, stdout_parts=parts)
    except Exception:
        return None
    trained = []
    for i, word_name in enumerate(words):
        sys.stdout.write(heads[i] + parts[i])
        A, B, pi = results[i]
        model = HMMTrained(states=n_states, symbols=len(centroids), A=A, B=B, Pi=pi, word=word_name)
        if model_dir is None:
            DataStorageHMM.save_hmm(model, print_messages=False)
        else:
            DataStorageHMM.save_hmm(model, base_dir=model_dir, print_messages=False)
        trained.append(model)
        print(f"Model saved for word: '{model.word}'")
    return trained


def train_hmm(show_progress=True, max_iterations=100, load_initial_params=False, base_dir="../Data",
              model_dir: Optional[str] = None, grouped: bool = True) -> Optional[List[HMMTrained]]:
    """Train one HMM per word (main.py:133-164); None on any error, as the reference."""
    print("Starting HMM training for all words...")
    try:
        centroids = load_mfcc_centroids(base_dir, print_messages=False)
        print(f"Loaded {len(centroids)} centroids")
        recordings_by_word = load_all_recordings_by_word(base_dir, purpose="TrainHMM", print_messages=False)
        print(f"Loaded recordings for {len(recordings_by_word)} words")
        trained = None
        if grouped:
            trained = _train_grouped(recordings_by_word, centroids, show_progress, max_iterations,
                                     load_initial_params, model_dir)
        if trained is None:  # word by word (the reference's loop, main.py:147-152)
            trained = []
            words = recordings_by_word.items()
        else:
            words = ()
        for word_name, word_recordings in words:
            print(f"\nTraining HMM for word: '{word_name}' with {len(word_recordings)} recordings")
            model = training_with_save(word_recordings, centroids, word_name, max_iterations=max_iterations,
                                       show_progress=show_progress, load_initial_params=load_initial_params,
                                       base_dir=model_dir)
            trained.append(model)
            print(f"Model saved for word: '{model.word}'")
        print("\nHMM training completed successfully!")
        print(f"Total models trained: {len(trained)}")
        print(f"Words trained: {[h.word for h in trained]}")
        return trained
    except Exception as e:  # the reference logs and returns None (main.py:162-164)
        logger.error(f"Error during HMM training: {e}")
        return None


def test(show_progress=False, base_dir="../Data", model_dir: Optional[str] = None):
    """Classify the Test recordings with the saved models (main.py:167-197); returns
    (true_labels, predicted_labels), or None when there is nothing to test."""
    print("Loading trained HMM models...")
    all_hmm = DataStorageHMM.load_all_hmms(base_dir=model_dir) if model_dir else DataStorageHMM.load_all_hmms()
    if not all_hmm:
        print("No trained HMM models found. Please train models first.")
        return None
    print(f"Loaded {len(all_hmm)} HMM models for words: {[h.word for h in all_hmm]}")
    test_recordings = load_all_recordings_by_word(base_dir, purpose="Test", print_messages=False)
    print(f"Loaded test recordings for {len(test_recordings)} words")
    trained_words = {h.word for h in all_hmm}
    filtered = {w: r for w, r in test_recordings.items() if w in trained_words}
    if not filtered:
        print("No test recordings found for trained words.")
        return None
    print(f"Testing on {len(filtered)} words: {list(filtered.keys())}")
    true_labels, predicted = test_hmm(all_hmm, filtered, base_dir=base_dir, show_progress=show_progress)
    return true_labels, predicted


def _cli(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("command", choices=["train", "test"])
    ap.add_argument("--data", default="../Data")
    ap.add_argument("--models", default=None, help="model directory (default: DataStorageHMM's)")
    # `python main.py train` runs train_hmm(show_progress=True, max_iterations=2) (HMM/main.py:268)
    ap.add_argument("--max-iterations", type=int, default=2)
    ap.add_argument("--load-initial-params", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    if a.command == "train":
        ok = train_hmm(show_progress=not a.quiet, max_iterations=a.max_iterations,
                       load_initial_params=a.load_initial_params, base_dir=a.data, model_dir=a.models)
        return 0 if ok is not None else 1
    res = test(base_dir=a.data, model_dir=a.models)
    if res is None:
        return 1
    t, p = res
    acc = sum(x == y for x, y in zip(t, p)) / max(len(t), 1)
    print(f"Accuracy: {100.0 * acc:.2f}% ({len(t)} recordings)")
    return 0


if __name__ == "__main__":
    raise SystemExit(_cli())
