"""Multi-process (gloo, world_size 2, CPU) test of the N>1 path: contiguous env shards keyed
by global env id, no data-path exchange, and the all-gather of episode summaries.  The
per-rank stepping here is the CPU oracle standing in for each rank's GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oc_testlib as tl
from gym_cooking_amd import dist as ocdist
from gym_cooking_amd import levels

from oracle import oracle

LEVEL, A, B_RANK, STEPS, SEED = "partial-divider_salad", 2, 3000, 130, 17


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_shard(env_offset, B):
    """Returns (final canonical planes, totals) of the oracle on global ids [off, off+B)."""
    ob = oracle.OracleBatch(levels.load_level(LEVEL), A, 100, B)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    tot = np.zeros(5, np.int64)
    for t in range(STEPS):
        ob.gen_actions(act, env_offset, t, SEED)
        fl_in = tl.planes_view(s, A, ob.K, ob.pitch)["fl"][:B].copy()
        coll = np.zeros(ob.pitch, np.uint8)
        ob.step(s, s2, act, None, coll)
        s, s2 = s2, s
        v = tl.planes_view(s, A, ob.K, ob.pitch)
        fl = v["fl"][:B]
        ended = ((fl_in & 1) == 0) & ((fl & 1) == 1)
        tot += np.array([ended.sum(), (ended & ((fl & 2) > 0)).sum(), v["t"][:B][ended].astype(np.int64).sum(),
                np.unpackbits(coll[:B]).sum(), (ended & ((fl & 4) > 0)).sum()], dtype=np.int64)
    return tl.env_view(s, A, ob.K, ob.pitch, B), tot


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    ocdist.init("gloo")
    sh = ocdist.shard(B_RANK, rank, world)
    planes, tot = _run_shard(sh.env_offset, sh.batch)
    gathered = ocdist.gather_summaries(torch.from_numpy(tot))
    t_max = ocdist.max_over_ranks(float(rank + 1), torch.device("cpu"))
    if rank == 0:
        q.put((gathered.numpy(), t_max))
    q.put((rank, planes))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_shards_and_summary_allgather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered, t_max = next(m for m in msgs if isinstance(m[0], np.ndarray))
    shards = dict(m for m in msgs if not isinstance(m[0], np.ndarray))
    assert t_max == 2.0
    # the two shards together are exactly one 2*B_RANK batch (global-id keyed RNG)
    full, tot_full = _run_shard(0, world * B_RANK)
    assert np.array_equal(np.concatenate([shards[0], shards[1]], axis=1), full)
    assert gathered.shape == (world, 5)
    assert np.array_equal(gathered.sum(0), tot_full)
    summ = ocdist.summarize(torch.from_numpy(gathered))
    assert summ["episodes"] == tot_full[0] > 0


def test_shard_arithmetic():
    assert [ocdist.shard(100, r, 4).env_offset for r in range(4)] == [0, 100, 200, 300]
    parts = [ocdist.shard_global(10, r, 3) for r in range(3)]
    assert [(p.env_offset, p.batch) for p in parts] == [(0, 4), (4, 3), (7, 3)]


def test_summarize_lists_device_ids():
    g = torch.tensor([[3, 1, 300, 2, 0, 0, 0x75, 0], [4, 2, 400, 1, 1, 0, 0x05, 0]], dtype=torch.int64)
    s = ocdist.summarize(g)
    assert s["episodes"] == 7 and s["successes"] == 3 and s["errors"] == 1
    assert s["per_rank_pci"] == ["0000:75:00", "0000:05:00"] and s["distinct_devices"] == 2
    assert "per_rank_pci" not in ocdist.summarize(g[:, :5])
