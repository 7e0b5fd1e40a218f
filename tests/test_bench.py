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
    cb = bench.cpu_baseline(8, 256, 200, "left_to_right", 0.5, 3, threads=2)
    assert cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0 and cb["unit"] == "utterances/s/iter"
    assert cb["ratio_vs_reference_8cores"] > 0 and cb["cpu_model"]


def test_bench_spawns_ranks_without_launcher():
    """`bench.py --gpus 2` with no torchrun: bench.py starts both ranks itself (127.0.0.1 rendezvous,
    nothing touching a GPU before the spawn) and rank 0 reports n_gpus 2 (dry run: no GPU here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--dry-run"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["sequences_per_gpu"] == 12_500 and d["config"]["workload"] == "cfg4"


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--dry-run"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_skewed_symbols_are_skewed_and_seeded():
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench
    u = bench.synthetic_symbols(500, 200, 8, 256, "U", 3)
    h = bench.synthetic_symbols(500, 200, 8, 256, "H", 3)
    assert h.dtype == np.int32 and h.min() >= 0 and h.max() < 256
    np.testing.assert_array_equal(h, bench.synthetic_symbols(500, 200, 8, 256, "H", 3))
    cu, ch = np.bincount(u, minlength=256), np.bincount(h, minlength=256)
    assert ch.max() > 4 * cu.max()  # hot symbols


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
    # algorithmic bytes per launch (24T + 16NT + 8 per sequence) over the launch time vs 8 TB/s
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["achieved"] == pytest.approx((24 * 200 + 16 * 8 * 200 + 8) * 10_000 / (rf["kernel_ms"] * 1e-3) / 1e9)
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"])
    # the tightest ceiling the counters measure: achieved / peak of one resource, so <= 1, with provenance
    bd = rf["bounds"]
    assert rf["binding"]["resource"] == bd["binding"] in ("hbm", "valu", "simd_valu", "cu_lds", "latency", "phase_model")
    assert 0 < rf["binding"]["frac"] <= 1.0
    assert rf["binding"]["frac"] == max(b["frac"] for b in bd.values() if isinstance(b, dict) and "frac" in b)
    # the busiest SIMD and CU on the engine's spread map: cfg3's 1,250 waves = 256 full workgroups + 113 of 2
    assert rf["launch_map"]["waves"] == 1250 and rf["launch_map"]["extra_waves"] == 2
    assert bd["waves_on_busiest_simd"] == 2 and bd["waves_on_busiest_cu"] == 6
    assert rf["kernel_src_sha16"] and d["cpu_baseline"]["value"] > 0


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


@pytest.mark.gpu
def test_bench_self_spawned_two_ranks_one_gpu_gloo():
    """`bench.py --gpus 2` without a launcher on the one-GPU box (both ranks on cuda:0, gloo carrying
    the all-reduce): the real E-step/all-reduce/M-step loop, n_gpus 2 in the line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "5", "--warmup", "1", "--R", "2000",
                        "--dist-backend", "gloo"], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["sequences_total"] == 4000
    assert d["comm"]["rccl_comm_ranks"] == 0 and d["synced"]["dropin_iterations"] == 20
    # gloo has no RCCL communicator: the engine's own peer all-reduce (IPC handles over gloo) runs the loop
    assert d["comm"]["kind"] == "peer" and d["comm"]["legs"]["peer"]["allreduce_us_per_iter"] > 0
    # without RCCL the peer leg is checked against the torch.distributed path before it may be the headline
    assert d["comm"]["legs_reference"] == "torch" and d["comm"]["legs_agree"]["peer"] is True


@pytest.mark.gpu
def test_bench_drops_a_peer_leg_that_disagrees():
    """The guard the first 8-GPU run depends on (hmm_training.py:503, L over all ranks): rank 1 pushes a wrong
    payload into the peer exchange (HMMBW_DIAG_PEER_PERTURB), so the peer leg's L trace disagrees with the
    torch.distributed reference; bench.py must drop the leg on every rank, report it in legs_failed, and still
    print a valid line timed on the torch path."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HMMBW_DIAG_PEER_PERTURB"] = "1:0.001"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "5", "--warmup", "1", "--R", "2000",
                        "--dist-backend", "gloo", "--no-cpu-baseline", "--no-synced"], cwd=ROOT, capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    c = d["comm"]
    assert "peer" in c["legs_failed"] and "differs" in c["legs_failed"]["peer"]
    assert c["legs_agree"] == {"peer": False, "torch": True} and c["legs_reference"] == "torch"
    assert c["kind"] == "torch" and "peer" not in c["legs"] and d["value"] > 0 and d["n_gpus"] == 2
    assert d["config"]["allreduce"].startswith("torch.distributed")


@pytest.mark.gpu
def test_bench_skewed_symbols_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "1", "--symbols", "H",
                        "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["config"]["symbols"] == "H" and d["value"] > 0


def test_engine_waves_on_the_spread_map():
    """The busiest SIMD and CU of the roofline bounds, counted on the engine's launch map (HMMBW_INFO_*):
    cfg3's 1,250 waves = 256 full workgroups + 113 of 2 active waves -> 6 waves on the busiest CU, 2 on its
    busiest SIMD; the cfg4 shard (1,563 waves, no spread) = 391 full workgroups -> 8 and 2."""
    sys.path.insert(0, ROOT)
    import bench
    cfg3 = {"waves": 1250, "workgroups": 369, "waves_per_workgroup": 4, "full_workgroups": 256, "extra_waves": 2,
            "work_queue": False}
    assert bench.engine_waves(10_000, 8, cfg3) == (1250, 2, 6)
    cfg4 = {"waves": 1563, "workgroups": 391, "waves_per_workgroup": 4, "full_workgroups": 391, "extra_waves": 4,
            "work_queue": False}
    assert bench.engine_waves(12_500, 8, cfg4) == (1563, 2, 8)
    assert bench.engine_waves(10_000, 8) == (1250, 2, 5)  # no map: pigeonhole
