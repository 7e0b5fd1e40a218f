"""On-disk formats either side of the path: the codebook and per-recording
frame JSON written by the reference's CodeVector pipeline.

* codevector.json: ``[{"mfcc": [...13], "id": k}, ...]`` (codevector_classes.py:321-342, 548-556)
* ``*_frames.json``: ``[{"raw_samples": [...], "mfcc_vector": [...13], ...}, ...]``
  (codevector_classes.py:251-279, 477-495).

Deviation (stated): the reference's RawDataMFCC.__post_init__ recomputes every frame's MFCC with
librosa (codevector_classes.py:217-224); librosa is not part of this build, so the stored
``mfcc_vector`` is used as-is.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import List

import numpy as np


@dataclass
class Centroid:
    mfcc: np.ndarray = field(default_factory=lambda: np.zeros(13))
    id: int = 0


@dataclass
class Frame:
    mfcc: np.ndarray
    frame_number: int = 0
    recording: str = ""


def load_centroids(path: str) -> List[Centroid]:
    with open(path) as fh:
        data = json.load(fh)
    return [Centroid(mfcc=np.asarray(d["mfcc"], dtype=np.float64).reshape(-1), id=d.get("id", i))
            for i, d in enumerate(data)]


def load_frames(path: str) -> List[Frame]:
    with open(path) as fh:
        data = json.load(fh)
    return [Frame(mfcc=np.asarray(d["mfcc_vector"], dtype=np.float64).reshape(-1),
                  frame_number=d.get("frame_number", 0), recording=d.get("recording", "")) for d in data]
