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


class BucketedNormGather:
    """The multi-rank step loop of bench.py: steps run in buckets of at most
    ``bucket`` steps; each bucket's device work (``launch(norms_rows, count)``: every step evaluates
    the shard and writes its own [max, sumsq] row) goes on ``stream`` and, with more than one rank,
    ONE asynchronous all-gather carries the bucket's rows (RCCL over xGMI on the GPU, gloo in the CPU
    tests).  Two norms buffers alternate, so the gather of bucket i overlaps bucket i + 1; before a
    buffer is overwritten (bucket i + 2) its pending gather is waited on — with RCCL, ``wait()``
    orders the current (launch) stream after the collective, so the next launch cannot overwrite
    rows the collective is still reading.

    launch(rows, count): writes rows[:count] (a [bucket, 2] float64 tensor); ``replay`` (optional,
    {(buffer, count): callable}) replaces launch with captured graphs of the same work.
    ``gather_always``: gather at one rank too (a one-rank process group: the RCCL path on one GPU)."""

    def __init__(self, world: int, bucket: int, device, launch, stream=None, replay=None, group=None,
                 gather_always: bool = False):
        import torch

        self.world, self.bucket, self.group = int(world), max(1, int(bucket)), group
        self.gather = self.world > 1 or bool(gather_always)
        self.launch, self.stream, self.replay = launch, stream, replay or {}
        self.norms = [torch.zeros(self.bucket, 2, dtype=torch.float64, device=device) for _ in range(2)]
        self.pending = [None, None]
        self.gathered = []  # (gathered rows [world * count, 2], count) per bucket, in issue order

    def sizes(self, steps: int):
        """Bucket sizes covering ``steps`` steps."""
        S = self.bucket
        return [S] * (steps // S) + ([steps % S] if steps % S else [])

    def _ctx(self):
        import contextlib

        import torch

        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def run_bucket(self, i: int, count: int):
        """Bucket i (count steps); returns the all-gather's work handle (None on one rank)."""
        j = i % 2
        with self._ctx():
            if self.pending[j] is not None:  # the gather of bucket i - 2 may still read norms[j]
                self.pending[j].wait()
                self.pending[j] = None
            fn = self.replay.get((j, count))
            if fn is not None:
                fn()
            else:
                self.launch(self.norms[j], count)
            if self.gather:
                out, work = all_gather_norms(self.norms[j][:count], group=self.group, async_op=True)
                self.pending[j] = work
                self.gathered.append((out, count))
                return work
        return None

    def run(self, steps: int):
        """All buckets of ``steps`` steps issued back to back; returns their work handles."""
        return [self.run_bucket(i, c) for i, c in enumerate(self.sizes(steps))]

    def reset(self):
        """Forget the gathered buckets (after the warm-up), keep nothing pending."""
        for j, w in enumerate(self.pending):
            if w is not None:
                w.wait()
            self.pending[j] = None
        self.gathered.clear()

    def last_bucket_report(self, rank: int, steps: int):
        """Checks on the last gathered bucket of a ``steps``-step run: every step's global norms
        (max over ranks, sum of squares over ranks) and whether this rank's gathered rows equal the
        rows it computed locally."""
        import torch

        last, cnt = self.gathered[-1]
        step_norms = combine_bucket(last, self.world, cnt)
        local = self.norms[(len(self.sizes(steps)) - 1) % 2][:cnt]
        mine = last.view(self.world, cnt, 2)[rank]  # rank-major [world * cnt, 2]
        return {"steps_in_last_bucket": cnt, "last_step_global_norms": list(step_norms[-1]),
                "local_rows_match": bool(torch.equal(mine.to(local.device), local))}
