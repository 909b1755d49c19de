"""Data-parallel path (bench.py --gpus N / trainer._allreduce_grads) on CPU with gloo, world 2.

The product path averages the flat gradient buffer with one collective per step before clip + Adam
(DDP semantics, per-replica BatchNorm); rank 0's weights are broadcast at start.  Here the
collectives run on CPU tensors (gloo) with the same trainer code that runs over RCCL on GPUs."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_q):
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gwn_amd import util
        from gwn_amd.engine import trainer
        torch.manual_seed(100 + rank)  # different init per rank: broadcast must unify them
        eng = trainer(util.StandardScaler(54.4, 19.5), 2, 12, 16, 16, 0.3, 1e-3, 1e-4, "cpu",
                      [torch.rand(16, 16), torch.rand(16, 16)], True, True, None, 4, 2)
        eng.broadcast_parameters(0)
        flat = eng.model._flat.clone()
        g = eng.optimizer.grad_flat
        g.copy_(torch.arange(g.numel(), dtype=torch.float32) * (rank + 1))
        eng._allreduce_grads()
        out_q.put((rank, flat.numpy().copy(), g.numpy().copy(), float(eng.model.bn[0].running_var.sum())))
    finally:
        torch.distributed.destroy_process_group()


def test_gloo_world2_broadcast_and_grad_average():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, flat, g, rv = q.get(timeout=300)
        res[r] = (torch.from_numpy(flat), torch.from_numpy(g), rv)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(res[0][0], res[1][0]), "parameters differ after broadcast"
    expect = torch.arange(res[0][1].numel(), dtype=torch.float32) * 1.5  # mean of (1x, 2x)
    assert torch.allclose(res[0][1], expect) and torch.allclose(res[1][1], expect)
    assert res[0][2] == res[1][2]


def _timing_worker(rank, world, port, out_q):
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["GWN_DIST_BACKEND"] = "gloo"
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        t, info = bench.rank_timing(1.0 + rank, world, rank, "cpu")
        out_q.put((rank, t, info))
    finally:
        torch.distributed.destroy_process_group()


def test_bench_rank_timing_gloo_world2():
    """bench.py's multi-rank record (SCALE lines): the timed region is the MAX over ranks, and the
    JSON carries the backend and world size torch.distributed saw plus the per-rank min / max."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, t, info = q.get(timeout=300)
        res[r] = (t, info)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        t, info = res[r]
        assert t == 2.0
        assert info == {"backend": "gloo", "world_seen": 2, "rank_seconds_min": 1.0, "rank_seconds_max": 2.0}
