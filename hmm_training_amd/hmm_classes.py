"""Model surface of the reference, kept byte-compatible: HMM/hmm_classes.py:7-95.

``HMMTrained`` holds one word model; ``DataStorageHMM`` writes/reads ``<base_dir>/<word>.json`` with
the keys {states, symbols, A, B, Pi, word} (``json.dump(..., indent=2)`` of ``ndarray.tolist()``),
so models trained here load in the reference and vice versa.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import List

import numpy as np


@dataclass(init=False)
class HMMTrained:
    """One trained word model (hmm_classes.py:7-23)."""

    states: int
    symbols: int
    A: np.ndarray
    B: np.ndarray
    Pi: np.ndarray
    word: str

    def __init__(self, states: int, symbols: int, A: np.ndarray, B: np.ndarray, Pi: np.ndarray, word: str):
        self.states, self.symbols = states, symbols
        self.A, self.B, self.Pi = A, B, Pi
        self.word = word

    def to_dict(self) -> dict:
        """JSON-ready dict, same key order as hmm_classes.py:25-34."""
        return {"states": self.states, "symbols": self.symbols, "A": self.A.tolist(), "B": self.B.tolist(),
                "Pi": self.Pi.tolist(), "word": self.word}

    @classmethod
    def from_dict(cls, data: dict) -> "HMMTrained":
        """Inverse of to_dict (hmm_classes.py:36-46); a missing key raises KeyError like the reference."""
        return cls(states=data["states"], symbols=data["symbols"], A=np.array(data["A"]), B=np.array(data["B"]),
                   Pi=np.array(data["Pi"]), word=data["word"])


class DataStorageHMM:
    """JSON persistence of HMMTrained (hmm_classes.py:48-95)."""

    @staticmethod
    def save_hmm(hmm: HMMTrained, base_dir: str = "../Data/ResultsHMM", print_messages: bool = True) -> None:
        os.makedirs(base_dir, exist_ok=True)
        path = os.path.join(base_dir, f"{hmm.word}.json")
        with open(path, "w") as fh:
            json.dump(hmm.to_dict(), fh, indent=2)
        if print_messages:
            print(f"Saved HMM for word '{hmm.word}' to {path}")

    @staticmethod
    def load_hmm(word: str, base_dir: str = "../Data/ResultsHMM", print_messages: bool = True) -> HMMTrained:
        path = os.path.join(base_dir, f"{word}.json")
        with open(path, "r") as fh:
            model = HMMTrained.from_dict(json.load(fh))
        if print_messages:
            print(f"Loaded HMM for word '{word}' from {path}")
        return model

    @staticmethod
    def load_all_hmms(base_dir: str = "../Data/ResultsHMM", print_messages: bool = True) -> List[HMMTrained]:
        models: List[HMMTrained] = []
        if not os.path.exists(base_dir):
            print(f"Directory {base_dir} does not exist")
            return models
        for name in os.listdir(base_dir):
            if not name.endswith(".json"):
                continue
            word = name[: -len(".json")]
            try:
                models.append(DataStorageHMM.load_hmm(word, base_dir, print_messages))
            except Exception as exc:  # the reference skips unreadable models (hmm_classes.py:87-91)
                print(f"Error loading HMM for word '{word}': {exc}")
        if print_messages:
            print(f"Loaded {len(models)} HMM models total")
        return models
