"""The entry-parallel eval kernel (cpl_kernels.hip cpl_eval_entry_kernel, tuning variant 5; the
default for 12+ contacts) against the pipelined / tile kernels, bit for bit, on every output (g, CSR Jacobian values, f, grad, fused residual
norms), and against the oracle: Ground and no-environment records of 1 ... 16 contacts, ragged
batches (tiles cut short), the degenerate x = 0 (0/0 cone entries: NaN positions must match)."""
import ctypes

import numpy as np
import pytest
import torch

import pyoracle
from centroidalplanner_amd import _abi
from centroidalplanner_amd.workload import generate, make_problem
from parity_util import check_outputs

CASES = [("ground", 1, 1), ("ground", 4, 1), ("ground", 4, 1001), ("ground", 8, 4097), ("ground", 16, 777),
         ("ground", 3, 130), ("none", 4, 513), ("none", 16, 65), ("none", 1, 2)]
OUTS = ("g", "jac", "f", "grad", "norms")


def _bits(t):
    return t.contiguous().view(torch.int64)


def _same_norms(a, b):
    """[max violation, sum of squares]: the max is exact; the sum's partials follow each kernel's
    tiles (a different summation order), equal to rounding."""
    a, b = a.cpu().numpy(), b.cpu().numpy()
    assert a[0] == b[0]
    assert a[1] == pytest.approx(b[1], rel=1e-12, abs=1e-300)


def _run(prob, xt, mt, variant):
    _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
    try:
        out = prob.eval_batch(xt, mt, outputs=OUTS)
        torch.cuda.synchronize()
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("env,N,B", CASES)
def test_entry_kernel_bitwise_default_and_oracle(env, N, B):
    prob = make_problem(N, env)
    x, mass, tag = generate(N, env, B, 977 + N)
    if B > 1:
        x[B // 2] = 0.0  # the cone's 0/0 entries (NaN) at one instance
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    ref = _run(prob, xt, mt, 2)  # the pipelined kernel (the tile kernel where x rows are not 16-byte aligned)
    got = _run(prob, xt, mt, 5)
    for k in ("g", "jac", "f", "grad"):
        assert torch.equal(_bits(got[k]), _bits(ref[k])), k
    _same_norms(got["norms"], ref["norms"])
    orc = pyoracle.eval_batch(prob.desc(), x, mass, tag)
    check_outputs(prob, env, x, {k: got[k].cpu().numpy() for k in ("g", "jac", "f", "grad")}, orc, tag)


@pytest.mark.gpu
def test_entry_kernel_large_batch_matches_pipe():
    """1,048,576 x 4 Ground (the north-star batch): the entry kernel's records equal the pipelined
    kernel's bit for bit (both checked against the oracle elsewhere)."""
    prob = make_problem(4, "ground")
    x, mass, _ = generate(4, "ground", 1 << 20, 5)
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    del x
    a = _run(prob, xt, mt, 2)
    b = _run(prob, xt, mt, 5)
    for k in ("g", "jac"):
        assert torch.equal(_bits(a[k]), _bits(b[k])), k
    _same_norms(a["norms"], b["norms"])


MIXED = [(4, 1001, "alternate"), (16, 777, "alternate"), (8, 515, "random"), (4, 64, "all_ground"),
         (4, 65, "all_sq"), (2, 1, "random"),
         # several partition blocks (PART_BLOCK = 1 024 instances): k_kind_write's cross-block offsets (the
         # exclusive prefix over the blocks' counts) and the last block's totals
         (4, 2049, "random"), (8, 5000, "alternate"), (4, 3073, "all_sq"), (2, 4100, "blocks")]


@pytest.mark.gpu
@pytest.mark.parametrize("N,B,pattern", MIXED)
def test_mixed_split_bitwise_default_and_oracle(N, B, pattern):
    """Mixed batches split by kind (variant 6: a stable partition of the instances by tag, the Ground
    ones through the entry kernel, the Superquadric ones through the Superquadric tile kernel, records
    written in place) equal the interleaved mixed kernel's bit for bit, and the oracle; degenerate
    lists (one kind only, a batch of one) included."""
    prob = make_problem(N, "mixed")
    x, mass, tag = generate(N, "mixed", B, 4242 + N)
    rng = np.random.default_rng(B)
    if pattern == "random":
        tag = rng.choice(np.array([1, 2], dtype=np.uint8), B)
    elif pattern == "all_ground":
        tag = np.full(B, 1, np.uint8)
    elif pattern == "all_sq":
        tag = np.full(B, 2, np.uint8)
    elif pattern == "blocks":  # runs of one kind across block boundaries: 1 500 Ground, 1 700 SQ, ...
        tag = np.where((np.arange(B) // 1500 + np.arange(B) // 1700) % 2 == 0, 1, 2).astype(np.uint8)
    x2, _, _ = generate(N, "superquadric", B, 4242 + N)  # Superquadric instances need points near the surface
    x = np.where((tag == 2)[:, None], x2, x)
    dev = torch.device("cuda:0")
    xt, mt, tt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev), torch.tensor(tag, device=dev)

    def run(variant):
        _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
        try:
            o = prob.eval_batch(xt, mt, tt, outputs=OUTS)
            torch.cuda.synchronize()
        finally:
            _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
        return o

    ref = run(3)  # the interleaved mixed tile kernel
    for variant in (0, 6, 7):  # the default, the kind split, the split with direct Jacobian rows
        got = run(variant)
        for k in ("g", "jac", "f", "grad"):
            assert torch.equal(_bits(got[k]), _bits(ref[k])), (variant, k)
        _same_norms(got["norms"], ref["norms"])
    orc = pyoracle.eval_batch(prob.desc(), x, mass, tag)
    check_outputs(prob, "mixed", x, {k: got[k].cpu().numpy() for k in ("g", "jac", "f", "grad")}, orc, tag)


@pytest.mark.gpu
def test_mixed_default_split_under_graph_capture():
    """The default mixed launch (the kind split: a stable partition, two kernels on two streams joined
    by events) inside a HIP graph: captured after one eager launch on the stream it replays the eager
    records bit for bit; captured on a fresh stream with no eager launch (the split's workspace and side
    stream do not exist yet, as in the solve engine's first iteration) the default falls back to the
    interleaved kernel — the same records, no capture error."""
    prob = make_problem(16, "mixed")
    x, mass, tag = generate(16, "mixed", 3001, 99)
    dev = torch.device("cuda:0")
    xt, mt, tt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev), torch.tensor(tag, device=dev)
    ref = prob.eval_batch(xt, mt, tt, outputs=("g", "jac"))
    torch.cuda.synchronize()
    for warm in (True, False):
        s = torch.cuda.Stream(dev)
        out = {"g": torch.empty_like(ref["g"]), "jac": torch.empty_like(ref["jac"])}
        with torch.cuda.stream(s):
            if warm:
                prob.eval_batch(xt, mt, tt, outputs=("g", "jac"), out=out, stream=s)
            s.synchronize()
            out["g"].zero_()
            out["jac"].zero_()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                prob.eval_batch(xt, mt, tt, outputs=("g", "jac"), out=out, stream=s)
            gr.replay()
        s.synchronize()
        for k in ("g", "jac"):
            assert torch.equal(_bits(out[k]), _bits(ref[k])), (warm, k)
