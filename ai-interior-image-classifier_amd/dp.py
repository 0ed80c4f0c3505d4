"""Whole-image data parallelism over the GPUs of one node (BASELINE.json config 3).

One process per GPU (torchrun / ``python -m torch.distributed.run``), weights replicated,
the global batch split into contiguous per-rank shards. Images are independent (no
cross-image op exists on the path), so the only exchange is the output
collection the north star names: one all-gather of the per-image logits ``[B/world, C]``
fp32 over RCCL/xGMI (backend "nccl" is RCCL on ROCm). With the ``gloo`` backend the same code
runs on CPU tensors (tests/test_dp.py).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def shard_bounds(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [start, stop) of rank; shards differ by at most one image."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def allgather_rows(local: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate every rank's equal-sized [b, ...] shard in rank order: [world*b, ...]."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    local = local.contiguous()
    if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local, group=group)
        return torch.cat(parts, dim=0)
    out = torch.empty((world * local.shape[0], *local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)  # RCCL over xGMI
    return out


def allgather_ragged(local: torch.Tensor, global_batch: int, group=None) -> torch.Tensor:
    """All-gather for shards of unequal size (pads to the largest shard, then trims)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    big = shard_bounds(global_batch, world, 0)[1]
    pad = torch.zeros((big, *local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    full = allgather_rows(pad, group)
    parts = [full[r * big: r * big + (lambda b: b[1] - b[0])(shard_bounds(global_batch, world, r))]
             for r in range(world)]
    return torch.cat(parts, dim=0)


class ShardedClassifier:
    """Per-rank engine + logits all-gather: ``classify_global`` returns the full [B, C] logits
    on every rank, rank r having computed rows shard_bounds(B, world, r)."""

    def __init__(self, engine, group=None):
        self.engine = engine
        self.group = group

    def classify_shard(self, local_pixels: torch.Tensor, out=None):
        return self.engine.classify(local_pixels, out)

    def classify_global(self, local_pixels: torch.Tensor, global_batch: int, out=None):
        res = self.engine.classify(local_pixels, out)
        return allgather_ragged(res.logits, global_batch, self.group), res
