"""The north-star point on the GPU: 1,048,576 instances x 4 contacts, Ground (BASELINE.json metric).

The bench times this size; these tests validate it, through the product path (the persistent
pipelined kernel at its full-size grid, every tile hand-off, the fused residual norms):
  * a strided sample of ~4k instances (plus the last one) against the oracle, bit for bit;
  * size-independent properties over ALL instances: the structural constants of the Jacobian
    (statics I3 rows, the Ground gradient (0, 0, 1), the normal block's zeros and ones) are exact,
    nothing is NaN at SURVEY.md §8(d) inputs, and the fused norms equal a full reduction of g;
  * past 2^31 output elements (13,000,000 instances: 2.26e9 Jacobian values, 18 GB), where 32-bit
    offsets would wrap: the instance record at b equals the record at b mod 1,048,576 for inputs
    tiled from the same 1M set.
"""
import numpy as np
import pytest

import pyoracle
from parity_util import check_outputs

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

B_NS = 1_048_576
N = 4


def _inputs():
    from centroidalplanner_amd.workload import CONFIGS, config_inputs

    return config_inputs(CONFIGS["ground4_1m"])


def _const_positions(prob):
    """(positions, values) of the Ground Jacobian's structural constants in the CSR values."""
    pos, val = list(range(3 * N)), [1.0] * (3 * N)           # statics rows 0-2: I3 per contact
    for k in range(N):
        jo = 6 + 15 * N + 27 * k
        pos += [jo, jo + 1, jo + 2]                           # EnvironmentConstraint p block
        val += [0.0, 0.0, 1.0]                                # src/Ground.cpp:33-34
        for r in range(3):                                    # EnvironmentNormal rows
            pos += [jo + 3 + 4 * r + c for c in range(4)]    # p block (src/Ground.cpp:49), n_r
            val += [0.0, 0.0, 0.0, 1.0]                       # src/Constraints/EnvironmentNormal.cpp:66-68
    return np.array(pos), np.array(val)


def test_north_star_full_size():
    prob, x, mass, _ = _inputs()
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    out = prob.eval_batch(xt, mt, outputs=("g", "jac", "norms"))
    torch.cuda.synchronize()
    assert out["jac"].shape == (B_NS, 174) and out["g"].shape == (B_NS, 30)

    # strided sample + the tail, bit-exact against the oracle
    idx = np.unique(np.concatenate([np.arange(0, B_NS, 251), [B_NS - 1]]))
    it = torch.as_tensor(idx, device=dev)
    got = {k: out[k][it].cpu().numpy() for k in ("g", "jac")}
    ref = pyoracle.eval_batch(prob.desc(), x[idx], mass[idx], outputs=("g", "jac"))
    rep = check_outputs(prob, "ground", x[idx], got, ref)
    assert rep["jac"]["bitwise_frac"] == 1.0 and rep["g"]["bitwise_frac"] == 1.0

    # properties over every instance
    pos, val = _const_positions(prob)
    cj = out["jac"][:, torch.as_tensor(pos, device=dev)]
    assert torch.equal(cj, torch.as_tensor(val, device=dev).expand_as(cj))
    assert not torch.isnan(out["jac"]).any() and not torch.isnan(out["g"]).any()
    _, _, gl, gu = prob.get_bounds_info()
    glt, gut = torch.as_tensor(gl, device=dev), torch.as_tensor(gu, device=dev)
    viol = torch.clamp(torch.maximum(glt - out["g"], out["g"] - gut), min=0.0)
    rn = out["norms"].cpu().numpy()
    assert rn[0] == float(viol.max())
    s = float((viol * viol).sum())
    assert abs(rn[1] - s) <= 1e-12 * s


def test_north_star_variants_agree():
    """Every kernel variant at the full size writes the same bits as the default launch."""
    from centroidalplanner_amd import _abi

    prob, x, mass, _ = _inputs()
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    base = prob.eval_batch(xt, mt, outputs=("g", "jac"))
    for variant in (1, 3):
        _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
        try:
            o = prob.eval_batch(xt, mt, outputs=("g", "jac"))
            torch.cuda.synchronize()
        finally:
            _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
        assert torch.equal(o["g"], base["g"]) and torch.equal(o["jac"], base["jac"]), variant
        del o


def test_beyond_int32_offsets():
    """13,000,000 instances: 2.26e9 Jacobian values (> 2^31), inputs tiled from the 1M set."""
    prob, x, mass, _ = _inputs()
    dev = torch.device("cuda:0")
    B = 13_000_000
    assert B * prob.nnz > 2 ** 31
    x1 = torch.tensor(x, device=dev)
    m1 = torch.tensor(mass, device=dev)
    reps = (B + B_NS - 1) // B_NS
    xt = x1.repeat(reps, 1)[:B].contiguous()
    mt = m1.repeat(reps)[:B].contiguous()
    del x1, m1
    out = prob.eval_batch(xt, mt, outputs=("g", "jac", "norms"))
    torch.cuda.synchronize()
    # the last 1M records (all past element 2^31 of jac) against the first 1M
    lo = B - B_NS
    src = torch.arange(lo, B, device=dev) % B_NS
    assert torch.equal(out["jac"][lo:], out["jac"][src])
    assert torch.equal(out["g"][lo:], out["g"][src])
    # and a strided sample of the high range against the oracle
    idx = np.arange(lo, B, 4099)
    ref = pyoracle.eval_batch(prob.desc(), x[idx % B_NS], mass[idx % B_NS], outputs=("g", "jac"))
    it = torch.as_tensor(idx, device=dev)
    assert np.array_equal(out["jac"][it].cpu().numpy(), ref["jac"])
    assert np.array_equal(out["g"][it].cpu().numpy(), ref["g"])


@pytest.mark.gpu
def test_bench_rccl_gather_path_on_one_gpu():
    """The multi-rank bench's collective path on real hardware with the one GPU a box has: a one-rank
    RCCL ("nccl") process group under torch.distributed.run, the bucketed asynchronous all-gather of
    the residual norms issued every bucket (`--collective-always`), the barriers and the max-over-ranks
    reduction — the calls an 8-GPU run makes, minus the peers.  The gathered rows must be the norms the
    rank computed, and the line must still be one JSON line."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "1", "--collective-always",
           "--config", "ground4", "--batch", "65536", "--steps", "23", "--warmup", "3", "--bucket", "5", "--no-pmc",
           "--no-cpu", "--no-side", "--no-check"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    ln = json.loads(lines[0])
    g = ln["residual_gather"]
    assert ln["n_gpus"] == 1 and ln["steps"] == 23 and g is not None
    assert g["steps_in_last_bucket"] == 3 and g["local_rows_match"]
    mx, ss = g["last_step_global_norms"]
    assert mx >= 0.0 and ss >= 0.0
