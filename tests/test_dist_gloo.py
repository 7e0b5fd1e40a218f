"""Multi-rank data-parallel path on CPU: world_size 2 (and 4) over torch.distributed gloo.

Each rank takes its contiguous length-balanced shard (engine.shard_bounds), computes its packed
statistics in the engine's layout (engine.StatsLayout) — here with the oracle standing in for the
E-step kernel, since there is no GPU — and the ranks all-reduce(sum) the buffer exactly as
BaumWelchEngine.enqueue_iterations does with RCCL.  The reduced buffer must equal the single-rank
statistics of the whole set, and the per-rank (m, s) log-likelihood slots must combine to the
global LSE_r log P_r of hmm_training.py:503.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT


def packed_stats(offsets, symbols, N, M, pi, A, B, world, rank):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from hmm_training_amd.engine import StatsLayout
    L = StatsLayout(N, M, world)
    buf = np.zeros(L.length)
    if len(offsets) > 1:
        s = O.estep_logstats(offsets, symbols, N, M, pi, A, B)
        buf[L.pi:L.pi + N] = np.exp(s.log_pi_num)
        buf[L.xi:L.xi + N * N] = np.exp(s.log_xi).reshape(-1)
        buf[L.gex:L.gex + N] = np.exp(s.log_gden_excl)
        buf[L.gall:L.gall + N] = np.exp(s.log_gden_all)
        buf[L.bnum:L.bnum + M * N] = np.exp(s.log_bnum).T.reshape(-1)
        lp = s.logP[np.isfinite(s.logP)]
        if lp.size:
            m = lp.max()
            buf[L.ll + 2 * rank] = m
            buf[L.ll + 2 * rank + 1] = np.exp(lp - m).sum()
    return buf, L


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from hmm_training_amd.engine import shard_bounds
        d = np.load(f"{GOLDEN}/bw_{case}.npz", allow_pickle=False)
        N, M = int(d["N"]), int(d["M"])
        off, sym = d["offsets"], d["symbols"]
        lengths = np.diff(off)
        lo, hi = shard_bounds(lengths, world)[rank]
        loff = off[lo:hi + 1] - off[lo]
        lsym = sym[off[lo]:off[hi]]
        buf, L = packed_stats(loff, lsym, N, M, d["init_pi"], d["init_A"], d["init_B"], world, rank)
        t = torch.from_numpy(buf)
        dist.all_reduce(t)  # the one collective per EM iteration
        np.save(os.path.join(out_dir, f"r{rank}.npy"), t.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, "n8_k256_cfg2"), (2, "zero_prob_seq"), (4, "n4_k16_default")])
def test_sharded_stats_allreduce_equals_single_rank(world, case, tmp_path, oracle):
    mp.start_processes(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    outs = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])  # every rank holds the same reduced buffer
    d = np.load(f"{GOLDEN}/bw_{case}.npz", allow_pickle=False)
    N, M = int(d["N"]), int(d["M"])
    full, L1 = packed_stats(d["offsets"], d["symbols"], N, M, d["init_pi"], d["init_A"], d["init_B"], 1, 0)
    from hmm_training_amd.engine import StatsLayout
    Lw = StatsLayout(N, M, world)
    red = Lw.decode(outs[0])
    ref = L1.decode(full)
    for key in ("pi_num", "xi", "gamma_den_excl", "gamma_den_all", "B_num"):
        np.testing.assert_allclose(red[key], ref[key], rtol=1e-12, atol=1e-300)
    # global convergence scalar from the per-rank slots == the reference's LSE over all log P
    lp = oracle.estep_logstats(d["offsets"], d["symbols"], N, M, d["init_pi"], d["init_A"], d["init_B"]).logP
    assert np.isclose(StatsLayout.lse_of_pairs(red["ll_pairs"]), oracle.lse(lp), rtol=1e-13)
    assert np.isclose(d["trace_L"][0], oracle.lse(lp), rtol=1e-12)


def _close_worker(rank, world, port, out_dir):
    """Rank 1 never reaches close() (it exits early): rank 0's bounded rendezvous must return False after its
    timeout instead of blocking; with both ranks present it returns True."""
    import sys
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, ROOT)
        from hmm_training_amd.engine import BaumWelchEngine

        class Fake:  # the rendezvous needs only the tag of the collective peer set-up and the group
            _group = None
        f = Fake()
        f._peer_tag = 1
        ok_all = BaumWelchEngine._close_rendezvous(f, 30.0)
        f._peer_tag = 2
        t0 = time.monotonic()
        ok_alone = BaumWelchEngine._close_rendezvous(f, 0.5) if rank == 0 else None
        dt = time.monotonic() - t0
        np.save(os.path.join(out_dir, f"c{rank}.npy"), np.array([ok_all, bool(ok_alone), dt]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_close_rendezvous_is_bounded(tmp_path):
    """BaumWelchEngine.close() with the peer all-reduce meets the other ranks before freeing its
    receive region; a rank that never arrives must not hold the others forever."""
    mp.start_processes(_close_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    c0, c1 = np.load(tmp_path / "c0.npy"), np.load(tmp_path / "c1.npy")
    assert c0[0] == 1 and c1[0] == 1      # both present: the rendezvous completes
    assert c0[1] == 0 and 0.4 < c0[2] < 10  # rank 1 absent: rank 0 gives up after its 0.5 s bound
