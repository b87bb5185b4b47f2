"""Batch-sharded multi-process path on CPU (gloo, world_size 2): shard ranges, the
max-over-ranks clock and the pooled-feature all-gather.  The encoder
itself needs the GPU; what is tested here is everything around it that differs at N>1."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from videomamba_amd.sharding import gather_pooled, max_over_ranks, shard_batch, shard_range


def test_shard_range_covers_batch_exactly():
    for n in (0, 1, 7, 32, 33):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = torch.arange(5 * 3, dtype=torch.float32).view(5, 1, 3)
        local = shard_batch(x, world, rank)
        # a rank-dependent "elapsed time": the max must be the slowest rank's
        t = max_over_ranks(1.0 + rank, torch.device("cpu"))
        pooled = gather_pooled(local * 2)
        q.put((rank, local.shape[0], t, pooled.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_clock_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    x = torch.arange(5 * 3, dtype=torch.float32).view(5, 1, 3)
    assert [o[1] for o in out] == [3, 2]          # 5 clips: ranks own 3 + 2
    assert all(o[2] == 2.0 for o in out)          # max over ranks
    for o in out:                                 # every rank sees the global pooled batch
        assert torch.equal(torch.tensor(o[3]), x * 2)
