"""Batch sharding across the GPUs of one node.

Clips are independent and each clip's streaming state stays with it, so the encoder
shards by batch with no collective on the data path.  One process per GPU
(torchrun: RANK / LOCAL_RANK / WORLD_SIZE); rank r owns the contiguous clip range
``shard_range(n, world, r)``.  The only collectives are off the data path:

* ``max_over_ranks``   — the timed interval's max (the bench's clock);
* ``gather_pooled``    — the optional all-gather of the pooled features
  ((B_local, 1, C) per rank; KB-sized, so one direct RCCL all-gather).
"""

from __future__ import annotations

import os
from typing import List, Tuple

import torch
import torch.distributed as dist


def dist_env() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1-process default)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``n`` clips owned by ``rank``; sizes differ by at most
    one clip and the lower ranks take the remainder."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_batch(x: torch.Tensor, world: int, rank: int) -> torch.Tensor:
    """This rank's slice of a global clip batch (dim 0)."""
    a, b = shard_range(x.shape[0], world, rank)
    return x[a:b]


def max_over_ranks(value: float, device: torch.device) -> float:
    """Max of a host scalar over all ranks (identity without a process group)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    # (gloo reduces host tensors: the multi-rank rehearsal on one GPU, and the CPU tests)
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_pooled(x_pool: torch.Tensor) -> torch.Tensor:
    """All-gather per-rank pooled features along dim 0 (ranks may hold different batch
    sizes).  Returns the global tensor in rank order."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x_pool
    world = dist.get_world_size()
    n = torch.tensor([x_pool.shape[0]], dtype=torch.int64, device=x_pool.device)
    sizes: List[torch.Tensor] = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    counts = [int(s.item()) for s in sizes]
    width = max(counts)
    pad = x_pool.new_zeros((width,) + tuple(x_pool.shape[1:]))
    pad[: x_pool.shape[0]] = x_pool
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous())
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
