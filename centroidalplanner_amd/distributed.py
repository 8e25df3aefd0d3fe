"""Multi-GPU execution of the batched callbacks: one process per GPU, instances sharded.

Instances are independent, so the batch is split into contiguous shards (one per rank) with no
data-path exchange.  The only collective is an all-gather of each shard's residual norms
[max violation, sum of squared violations] (cpl_residual_norms), RCCL over xGMI with the "nccl"
backend on ROCm, gloo on CPU in tests; it is issued asynchronously so it overlaps the next
evaluation, and one collective can carry a bucket of steps' norms.  (BASELINE.json north_star)
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


def combine_bucket(gathered, world: int, steps: int):
    """A gathered bucket (rank-major [world, steps, 2], flat or shaped) -> per-step global (max, sumsq)."""
    import numpy as np

    a = np.asarray(gathered.cpu() if hasattr(gathered, "cpu") else gathered, dtype=np.float64).reshape(world, steps, 2)
    return [(float(a[:, s, 0].max()), float(a[:, s, 1].sum())) for s in range(steps)]


def all_gather_norms(local_norms, group=None, async_op: bool = False):
    """All-gather per-shard norms (RCCL or gloo): a [2] tensor -> [2*world], or a bucket of steps
    [S, 2] (one row per step) -> [world*S, 2], rank-major — one collective for S steps."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    shape = (world * local_norms.shape[0],) + tuple(local_norms.shape[1:])  # [2*world] or [world*S, 2]
    out = torch.empty(shape, dtype=local_norms.dtype, device=local_norms.device)
    work = dist.all_gather_into_tensor(out, local_norms.contiguous(), group=group, async_op=async_op)
    return out, work
