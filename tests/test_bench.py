"""bench.py contract: one JSON line with the driver's fields plus roofline and cpu_baseline."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_cpu_baseline_sample_is_bounded():
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline(8, 256, 200, "left_to_right", 0.5, 3)
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0 and cb["unit"] == "utterances/s/iter"


@pytest.mark.gpu
def test_bench_single_gpu_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "10", "--warmup", "2", "--cpu-seconds", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 10 and d["value"] > 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1.5
    assert d["cpu_baseline"]["value"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu_gloo():
    """The N>1 code path of bench.py (launcher env, per-rank shards, max-over-ranks timing) with two
    ranks sharing the box's GPU; gloo stands in for RCCL, which needs one GPU per rank."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "5", "--warmup", "1",
           "--R", "2000", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["cpu_baseline"] is None
    assert d["config"]["parallelism"] == "dp2"
