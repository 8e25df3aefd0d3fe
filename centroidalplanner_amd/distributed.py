"""Multi-GPU execution of the batched callbacks: one process per GPU, instances sharded.

Instances are independent, so the batch is split into contiguous shards (one per rank) with no
data-path exchange.  The only collective is an all-gather of each shard's residual norms
[max violation, sum of squared violations] (cpl_residual_norms), RCCL over xGMI with the "nccl"
backend on ROCm, gloo on CPU in tests; it is issued asynchronously so it overlaps the next
evaluation.  (BASELINE.json north_star)
"""
from __future__ import annotations

from typing import Tuple


def shard(batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard (start, count) of ``batch`` instances for ``rank`` of ``world``; sizes differ by <= 1."""
    if world < 1 or not 0 <= rank < world or batch < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def combine_norms(gathered):
    """Per-rank [max, sumsq] rows (tensor/array [world, 2] or flat [2*world]) -> global (max, sumsq)."""
    import numpy as np

    a = np.asarray(gathered.cpu() if hasattr(gathered, "cpu") else gathered, dtype=np.float64).reshape(-1, 2)
    return float(a[:, 0].max()), float(a[:, 1].sum())


def all_gather_norms(local_norms, group=None, async_op: bool = False):
    """All-gather a [2] tensor of per-shard norms into a [2*world] tensor (RCCL or gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = torch.empty(2 * world, dtype=local_norms.dtype, device=local_norms.device)
    work = dist.all_gather_into_tensor(out, local_norms.contiguous(), group=group, async_op=async_op)
    return out, work
