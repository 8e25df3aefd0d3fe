"""Multi-process (world_size 2, gloo on CPU) test of the sharded path: each rank evaluates its
contiguous shard of one seeded batch (here through the oracle: the CPU stands in for the rank's GPU),
computes its shard's residual norms, and the all-gather + combine must reproduce the norms of the
whole batch; the shards must tile the batch exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from centroidalplanner_amd.distributed import combine_norms, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _norms(g, gl, gu):
    viol = np.maximum(np.maximum(gl - g, g - gu), 0.0)
    viol = np.where(np.isnan(g), np.inf, viol)
    return np.array([viol.max(initial=0.0), (viol ** 2).sum()])


def _worker(rank, world, port, batch, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import pyoracle
    import torch.distributed as dist

    from centroidalplanner_amd.distributed import all_gather_norms
    from centroidalplanner_amd.workload import generate, make_problem

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = make_problem(4, "ground")
    x, mass, _ = generate(4, "ground", batch, 2024)
    start, count = shard(batch, rank, world)
    g = pyoracle.eval_batch(prob.desc(), x[start:start + count], mass[start:start + count], outputs=("g",),
                            nthreads=1)["g"]
    _, _, gl, gu = prob.get_bounds_info()
    local = torch.tensor(_norms(g, gl, gu), dtype=torch.float64)
    out, work = all_gather_norms(local, async_op=True)
    work.wait()
    q.put((rank, start, count, out.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("batch", [1001, 64])
def test_sharded_norms_gloo_world2(batch):
    import pyoracle
    from centroidalplanner_amd.workload import generate, make_problem

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert sum(r[2] for r in res) == batch and res[0][1] == 0 and res[1][1] == res[0][2]
    assert np.array_equal(res[0][3], res[1][3])  # every rank sees the same gathered vector
    gmax, gsum = combine_norms(res[0][3])
    prob = make_problem(4, "ground")
    x, mass, _ = generate(4, "ground", batch, 2024)
    g = pyoracle.eval_batch(prob.desc(), x, mass, outputs=("g",), nthreads=1)["g"]
    _, _, gl, gu = prob.get_bounds_info()
    full = _norms(g, gl, gu)
    assert gmax == full[0]
    assert gsum == pytest.approx(full[1], rel=1e-12)


def test_shard_tiles_batch():
    for batch in (0, 1, 7, 65536, 1048577):
        for world in (1, 2, 3, 8):
            got = [shard(batch, r, world) for r in range(world)]
            assert got[0][0] == 0
            assert all(got[r][0] + got[r][1] == got[r + 1][0] for r in range(world - 1))
            assert got[-1][0] + got[-1][1] == batch
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def _bucket_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from centroidalplanner_amd.distributed import all_gather_norms

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bucket = torch.tensor([[10.0 * rank + s, 100.0 * rank + s] for s in range(3)], dtype=torch.float64)
    out, work = all_gather_norms(bucket, async_op=True)  # one collective for a bucket of 3 steps
    work.wait()
    q.put((rank, out.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_norms_gloo_world2():
    """bench.py's bucketed gather: one all-gather carries S steps' norms, rank-major; combine_bucket
    recovers every step's global (max, sumsq)."""
    from centroidalplanner_amd.distributed import combine_bucket

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1])
    steps = combine_bucket(res[0][1], world, 3)
    assert steps == [(10.0 + s, (0.0 + s) + (100.0 + s)) for s in range(3)]


def _loop_worker(rank, world, port, steps, bucket, q):
    """The bench's bucketed step loop (distributed.BucketedNormGather, the code bench.py runs on
    N GPUs) under gloo: every step writes synthetic per-rank norms rows; the handles are waited in
    REVERSE issue order (out-of-order completion), then the gathered buckets are checked."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist

    from centroidalplanner_amd.distributed import BucketedNormGather, combine_bucket

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    step_no = [0]
    written = []

    def launch(rows, count):  # stands in for `count` eval steps writing their [max, sumsq] rows
        for s in range(count):
            k = step_no[0]
            rows[s, 0] = 10.0 * rank + k       # max violation of this rank's shard at step k
            rows[s, 1] = 1.0 + rank + 0.5 * k  # sum of squares
            written.append((k, rows[s].clone()))
            step_no[0] += 1

    run = BucketedNormGather(world, bucket, torch.device("cpu"), launch)
    for w in run.run(3):  # warm-up buckets, then forgotten
        if w is not None:
            w.wait()
    run.reset()
    step_no[0] = 0
    written.clear()
    works = run.run(steps)
    for w in reversed(works):
        if w is not None:
            w.wait()
    report = run.last_bucket_report(rank, steps)
    per_step = []
    for out, cnt in run.gathered:
        per_step += combine_bucket(out, world, cnt)
    q.put((rank, [c for _, c in run.gathered], per_step, report))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("steps,bucket", [(23, 10), (4, 10), (9, 1)])
def test_bucketed_gather_loop_gloo_world2(steps, bucket):
    """Every timed step's norms reach every rank, combined per step (max over ranks, sum over ranks);
    the last bucket's own rows match what the rank computed; bucket sizes cover the steps."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loop_worker, args=(r, world, port, steps, bucket, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, per_step, report in res:
        assert sum(counts) == steps and all(c <= bucket for c in counts)
        assert len(per_step) == steps
        for k, (gmax, gsum) in enumerate(per_step):
            assert gmax == 10.0 * (world - 1) + k
            assert gsum == sum(1.0 + r + 0.5 * k for r in range(world))
        assert report["local_rows_match"]
        assert report["steps_in_last_bucket"] == counts[-1]
    assert res[0][2] == res[1][2]
