"""hmm_training_amd — MI355X-native Baum-Welch trainer for discrete HMMs.

Drop-in for DemianMArin/HMM_Training's HMM/hmm_training.py, hmm_classes.py and hmm_testing.py;
the EM hot path runs in hand-written gfx950 HIP kernels behind the C ABI of include/hmmbw.h.
"""
from .hmm_classes import DataStorageHMM, HMMTrained  # noqa: F401

__all__ = ["HMMTrained", "DataStorageHMM", "hmm_training", "training_with_save", "get_observations",
           "calculate_log_likelihood", "BaumWelchEngine"]


def __getattr__(name):
    # the engine-backed entry points load libhmmbw.so (and torch) lazily
    if name in ("hmm_training", "training_with_save", "get_observations", "safe_log", "safe_exp", "log_sum_exp"):
        from . import hmm_training as _ht
        return getattr(_ht, name)
    if name in ("calculate_log_likelihood", "score_matrix", "test_hmm"):
        from . import hmm_testing as _te
        return getattr(_te, name)
    if name == "BaumWelchEngine":
        from .engine import BaumWelchEngine
        return BaumWelchEngine
    raise AttributeError(name)
