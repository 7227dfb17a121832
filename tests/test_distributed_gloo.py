"""World-size-2 gloo test of the date-sharded gather used by Backtest.run / bench.py."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from porqua_amd.backtest import gather_shards, shard_range


def _worker(rank, world, port, total, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard_range(total, rank, world)
    W = np.arange(s, e)[:, None] * 10.0 + np.arange(n)[None, :]
    ST = np.full(e - s, 1, dtype=np.int32)
    ST[::3] = 2
    OBJ = np.arange(s, e) * 0.5
    Wf, STf, Of = gather_shards(W, ST, OBJ, total, world, dist, torch.device("cpu"))
    ok = (Wf.shape == (total, n) and np.array_equal(Wf, np.arange(total)[:, None] * 10.0 + np.arange(n)[None, :])
          and np.array_equal(Of, np.arange(total) * 0.5) and len(STf) == total)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_shards_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 2000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 11, 5, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def _agree_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from porqua_amd.backtest import agree_all
    # only rank 1's shard cannot batch (e.g. unequal window lengths in one of its chunks):
    # every rank must fall back together instead of rank 0 blocking in the all-gather
    a = agree_all(rank != 1, dist, torch.device("cpu"))
    b = agree_all(True, dist, torch.device("cpu"))
    q.put((rank, a, b))
    dist.barrier()
    dist.destroy_process_group()


def test_batchability_is_agreed_by_all_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 2000
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, False, True), (1, False, True)]
