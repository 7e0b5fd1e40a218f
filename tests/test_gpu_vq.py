"""GPU parity of the HIP VQ encoder (hmmbw_vq_encode) that replaces get_observations,
HMM/hmm_training.py:82-120: indices bit-identical to the reference's golden vectors and to the oracle
(itself pinned bit for bit to np.linalg.norm, tests/test_oracle_golden.py), winning distances
bit-identical to the oracle's."""
import os
from types import SimpleNamespace as NS

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")


def test_get_observations_matches_reference_golden():
    from hmm_training_amd.hmm_training import get_observations
    d = np.load(os.path.join(GOLDEN, "vq_k64.npz"), allow_pickle=False)
    off = d["offsets"]
    recs = [[NS(mfcc=f) for f in d["frames"][off[i]:off[i + 1]]] for i in range(len(off) - 1)]
    out = get_observations(recs, [NS(mfcc=c) for c in d["centroids"]])
    assert all(o.dtype == np.int64 for o in out)
    assert np.array_equal(np.concatenate(out), d["symbols"])


def tricky(rng, F, K, D=13):
    cents = rng.normal(size=(K, D)) * rng.uniform(0.5, 20.0, size=(K, 1))
    frames = rng.normal(size=(F, D)) * 8.0
    n = min(F // 4, 500)
    frames[:n] = cents[rng.integers(0, K, size=n)] + 1e-9 * rng.normal(size=(n, D))
    frames[n + 1, 1:] = np.nan
    frames[n + 3, 1:] = np.inf
    if K >= 4:
        cents[K - 1] = cents[1]                   # duplicate: 1 must win over K - 1
        frames[n] = 0.5 * (cents[2] + cents[3])   # (near-)equidistant
        frames[n + 2] = cents[1]
    return frames, cents


@pytest.mark.parametrize("F,K,D", [(5000, 256, 13), (777, 64, 13), (1000, 100, 21), (300, 5, 4), (64, 1, 13)])
def test_vq_matches_oracle_bitwise(oracle, F, K, D):
    from hmm_training_amd.hmm_training import vq_encode
    rng = np.random.default_rng(F + K + D)
    frames, cents = tricky(rng, F, K, D)
    idx, dist = vq_encode(frames, cents, return_distances=True)
    ridx, rdist = oracle.vq(frames, cents, return_dist=True)
    assert np.array_equal(idx, ridx)
    assert np.array_equal(dist.view(np.int64), rdist.view(np.int64))


def test_vq_full_size_sampled(oracle):
    """cfg3 scale: 2M frames (10,000 utterances x 200) x 256 centroids; a sample against the oracle."""
    from hmm_training_amd.hmm_training import vq_encode
    rng = np.random.default_rng(7)
    cents = rng.normal(size=(256, 13)) * 4.0
    frames = cents[rng.integers(0, 256, size=2_000_000)] + rng.normal(size=(2_000_000, 13))
    idx = vq_encode(frames, cents)
    pick = rng.choice(len(frames), size=4000, replace=False)
    assert np.array_equal(idx[pick], oracle.vq(frames[pick], cents))
    assert idx.min() >= 0 and idx.max() < 256


def test_vq_edge_cases():
    from hmm_training_amd.hmm_training import get_observations
    assert get_observations([[], []], [NS(mfcc=np.zeros(13))]) [0].size == 0
    out = get_observations([[NS(mfcc=np.ones(13))] * 3], [])
    assert np.array_equal(out[0], [0, 0, 0])
    with pytest.raises(ValueError):
        get_observations([[NS(mfcc=np.ones(13))]], [NS(mfcc=np.ones(7))])
