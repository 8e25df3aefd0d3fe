"""bench.py's multi-rank launch on the CPU: `python bench.py --gpus 2` with no WORLD_SIZE spawns two
rank processes itself (the driver's 8-GPU line is the same code with RCCL), rehearsed here with gloo
and the shard's norms from the oracle (tests/bench_rehearsal_stub.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "bench_rehearsal_stub.py")
BASE = ["--rehearse-cpu", STUB, "--steps", "7", "--warmup", "2", "--bucket", "3", "--no-pmc", "--no-cpu",
        "--no-side", "--no-check"]


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.lstrip().startswith("{")]


@pytest.mark.parametrize("config,batch", [("ground4", 2048), ("mixed16", 1001)])
def test_spawned_world2_prints_one_line(config, batch):
    r = _run(["--gpus", "2", "--config", config, "--batch", str(batch)] + BASE)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["steps"] == 7 and ln["warmup"] == 2
    assert ln["residual_gather"]["local_rows_match"] is True
    assert ln["residual_gather"]["steps_in_last_bucket"] == 1  # 7 steps in buckets of 3
    assert ln["config"]["batch_total"] == 2 * batch  # --batch: a per-rank batch, weak scaling
    assert ln["scaling"] == "weak"


def test_config4_shards_the_node_batch():
    """configs[3] is quoted as one batch over the node: without --batch each rank takes a shard and the
    line says strong scaling."""
    from centroidalplanner_amd.distributed import shard

    r = _run(["--gpus", "2", "--config", "mixed16"] + BASE, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    (ln,) = _json_lines(r.stdout)
    assert ln["scaling"] == "strong"
    assert ln["config"]["batch_total"] == 1048576
    assert ln["config"]["batch_per_gpu"] == shard(1048576, 0, 2)[1]


def test_single_rank_needs_no_spawn():
    r = _run(["--config", "ground4", "--batch", "512"] + BASE)
    assert r.returncode == 0, r.stderr[-2000:]
    (ln,) = _json_lines(r.stdout)
    assert ln["n_gpus"] == 1 and ln["residual_gather"] is None


def test_gpus_disagreeing_with_world_size_is_refused():
    r = _run(["--gpus", "4", "--config", "ground4", "--batch", "64"] + BASE,
             env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr
    assert not _json_lines(r.stdout)


def test_a_failing_rank_fails_the_launch():
    r = _run(["--gpus", "2", "--config", "ground4", "--batch", "64"] + BASE,
             env_extra={"CPL_REHEARSAL_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr
    assert not _json_lines(r.stdout)
