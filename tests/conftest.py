import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden_cases():
    return sorted(f[3:-4] for f in os.listdir(GOLDEN) if f.startswith("bw_") and f.endswith(".npz"))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.load()
    return O


def host_threads() -> int:
    """CPU threads this process may use (the GPU box exposes a 16-thread share of a larger machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(n, 16))


@pytest.fixture()
def oracle_mt(oracle):
    """The oracle with OpenMP over utterances (same terms, per-thread accumulators merged in thread
    order: equal to the serial restatement to ~1e-12), for full-size comparisons; serial again after."""
    oracle.set_threads(host_threads())
    yield oracle
    oracle.set_threads(1)
