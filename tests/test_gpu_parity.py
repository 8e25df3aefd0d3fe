"""GPU parity: the HIP path (through the C-ABI) against the oracle on the same seeded inputs.

Bit-exact for every entry that carries no data-dependent pow; within 1e-10 (conditioning-aware for
the normal-Jacobian diagonals) for Superquadric pow-bearing entries — see tests/parity_util.py.
"""
import numpy as np
import pytest

import pyoracle
from parity_util import check_outputs

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

OUTPUTS = ("g", "jac", "f", "grad")


def _run(prob, x, mass=None, tag=None, outputs=OUTPUTS):
    from centroidalplanner_amd import ENV_SUPERQUADRIC

    dev = torch.device("cuda:0")
    xt = torch.tensor(x, device=dev)
    mt = None if mass is None else torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    out = prob.eval_batch(xt, mt, tt, outputs=outputs)
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    ref = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=outputs)
    return got, ref


def _check(prob, env, x, got, ref, tag=None):
    return check_outputs(prob, env, x, got, ref, tag)


@pytest.mark.parametrize("env", ["ground", "none", "superquadric", "mixed"])
@pytest.mark.parametrize("N", [1, 4, 8, 12, 16])
def test_parity_configs(env, N):
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    B = 777  # ragged: 12 full tiles + a partial one
    x, mass, tag = generate(N, env, B, 1000 + N)
    got, ref = _run(prob, x, mass, tag)
    _check(prob, env, x, got, ref, tag)


@pytest.mark.parametrize("B", [1, 63, 64, 65, 129])
def test_parity_ragged_batches(B):
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(4, "ground")
    x, mass, tag = generate(4, "ground", B, B)
    got, ref = _run(prob, x, mass, tag)
    _check(prob, "ground", x, got, ref)


def test_parity_default_mass_and_subsets():
    """mass=None uses the template mass; any output subset may be requested."""
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(4, "ground", mass=73.5)
    x, _, _ = generate(4, "ground", 100, 5)
    for outs in (("g",), ("jac",), ("f",), ("grad",), ("g", "f")):
        got, ref = _run(prob, x, None, None, outputs=outs)
        for k in outs:
            assert np.array_equal(got[k], ref[k], equal_nan=True), k


def test_parity_degenerate_points():
    """NaN positions: x = 0 (IPOPT start), F = 0, p_k = C_k on the superquadric."""
    from centroidalplanner_amd.workload import make_problem

    for env in ("ground", "none", "superquadric"):
        prob = make_problem(4, env)
        n = prob.n
        x = np.zeros((5, n))
        x[1] = 0.3
        x[2, 3:6] = 0.0                         # F = 0 for contact1
        x[2, 6:9] = [0.0, 0.0, 1.0]             # p = C
        x[2, 9:12] = [0.0, 0.0, 1.0]
        x[3] = np.linspace(-1, 1, n)
        x[4, 6:9] = [0.0, 0.05, 1.0]            # p_x = C_x
        got, ref = _run(prob, x, np.full(5, 100.0))
        for k in got:
            assert np.array_equal(np.isnan(got[k]), np.isnan(ref[k])), (env, k)
        if env != "superquadric":
            for k in got:
                assert np.array_equal(got[k], ref[k], equal_nan=True), (env, k)
        assert np.isnan(ref["jac"]).any()


def test_parity_superquadric_stress_box():
    """Full box, including points within 1e-3 of the centre planes (ill-conditioned diagonals).
    Beyond the policy of parity_util, on the PLAIN relative error: the Jacobian's pow-bearing entries
    off the normal-Jacobian diagonals within 1e-10 (asserted); the diagonals and the g entries (both
    with cancelling expressions: the expanded (C - p)^2 numerators, sum pow - 1 and n - n_env) graded
    on the plain 1e-10 bound wherever |ref| is above the rounding noise of their un-cancelled terms —
    the diagonals all inside it (asserted), the g entries outside it counted, with their errors in ulps
    of the un-cancelled terms (near the surface a one-ulp difference of a power of magnitude ~1 is a
    large part of |sum pow - 1|).  The histograms go to gpurun_out/sq_stress_hist.json."""
    import json
    import os

    from parity_util import RTOL, plain_rel_diagonals, plain_rel_g_graded, plain_rel_off_diagonals

    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(8, "superquadric")
    x, mass, tag = generate(8, "superquadric", 20000, 99, stress=True)
    got, ref = _run(prob, x, mass, tag)
    _check(prob, "superquadric", x, got, ref)
    off = plain_rel_off_diagonals(prob, "superquadric", x, got, ref)
    diag = plain_rel_diagonals(prob, "superquadric", x, got, ref)
    gg = plain_rel_g_graded(prob, "superquadric", x, got, ref)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "sq_stress_hist.json"), "w") as fh:
        json.dump({"instances": int(x.shape[0]), "contacts": 8, "plain_off_diagonal": off, "plain_diagonal": diag,
                   "plain_g_graded": gg}, fh, indent=1, sort_keys=True)
    assert off["jac"] <= RTOL, off
    assert diag["outside"] == 0, diag
    # the g entries past the plain bound: few, and each a last-ulp difference of the un-cancelled terms
    assert gg["outside"] <= 1e-5 * gg["graded"], gg
    assert all(u <= 4.0 for u in gg["outside_err_ulps"]), gg


def test_parity_contact_names_order():
    """Arbitrary names: variables follow the vector order, constraints the std::map order."""
    from centroidalplanner_amd import CplProblem, Ground
    from centroidalplanner_amd.workload import generate

    env = Ground()
    env.SetGroundZ(0.05)
    env.SetMu(0.7)
    names = ["r_foot", "l_foot", "Hand", "arm_10", "arm_2", "zeta"]
    prob = CplProblem(names, 80.0, env)
    prob.SetManipulationWrench([1, 2, 3, 4, 5, 6])
    prob.SetForceThreshold("l_foot", 20.0)
    prob.SetContactPosWeight("arm_2", 3.0)
    prob.SetForceRef("zeta", [1.0, -2.0, 30.0])
    prob.SetCoMRef([0.1, 0.0, 0.9])
    prob.SetCoMWeight(2.0)
    x, mass, _ = generate(len(names), "ground", 300, 11)
    got, ref = _run(prob, x, mass)
    _check(prob, "ground", x, got, ref)


def test_residual_norms_match_host():
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(4, "ground")
    x, mass, _ = generate(4, "ground", 5000, 3)
    dev = torch.device("cuda:0")
    out = prob.eval_batch(torch.tensor(x, device=dev), torch.tensor(mass, device=dev), outputs=("g",))
    rn = prob.residual_norms(out["g"]).cpu().numpy()
    g = pyoracle.eval_batch(prob.desc(), x, mass, outputs=("g",))["g"]
    _, _, gl, gu = prob.get_bounds_info()
    viol = np.maximum(np.maximum(gl - g, g - gu), 0.0)
    assert rn[0] == viol.max()
    assert abs(rn[1] - (viol ** 2).sum()) <= 1e-9 * (viol ** 2).sum()


@pytest.mark.parametrize("variant,lds_kb,wg,nt", [(1, 64, 256, 0), (3, 16, 128, 1), (3, 160, 256, 0), (3, 8, 128, 0),
                                                  (2, 32, 256, 1), (2, 64, 256, 0), (2, 8, 256, 1), (0, 0, 256, 1)])
@pytest.mark.parametrize("env,N", [("ground", 4), ("superquadric", 8), ("mixed", 16), ("none", 3)])
def test_parity_kernel_variants(variant, lds_kb, wg, nt, env, N):
    """Every kernel variant / tile size gives the same results (tile sizes 8..64, odd records)."""
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    x, mass, tag = generate(N, env, 333, 77 + N)
    _abi.check(_abi.lib.cpl_set_tuning(variant, lds_kb, wg, nt, 0))
    try:
        got, ref = _run(prob, x, mass, tag)
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    _check(prob, env, x, got, ref, tag)


@pytest.mark.parametrize("env,N,B", [("ground", 4, 100003), ("superquadric", 8, 40001), ("mixed", 16, 20011)])
def test_parity_pipelined_many_tiles(env, N, B):
    """The persistent pipelined kernel (variant 2) walks many tiles per workgroup through its double
    buffer; a batch far above the resident grid exercises every buffer hand-off and the odd tail."""
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    x, mass, tag = generate(N, env, B, 991 + N)
    _abi.check(_abi.lib.cpl_set_tuning(2, 32, 256, 1, 0))
    try:
        got, ref = _run(prob, x, mass, tag)
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    _check(prob, env, x, got, ref, tag)


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("env,N,B", [("ground", 4, 70001), ("none", 4, 5000), ("superquadric", 8, 3001),
                                     ("mixed", 16, 2003), ("ground", 4, 1)])
def test_fused_residual_norms(variant, env, N, B):
    """cpl_eval_batch_norms: the norms reduced inside the eval launch equal the host reduction of
    the oracle's g; g / jac are unchanged; repeated launches give bit-identical norms."""
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    x, mass, tag = generate(N, env, B, 4242 + N)
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
    try:
        out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
        n1 = out["norms"].clone()
        out2 = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
        torch.cuda.synchronize()
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    assert torch.equal(n1, out2["norms"])
    ref = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=("g", "jac"))
    got = {"g": out["g"].cpu().numpy(), "jac": out["jac"].cpu().numpy()}
    _check(prob, env, x, got, ref, tag)
    _, _, gl, gu = prob.get_bounds_info()
    viol = np.maximum(np.maximum(gl - got["g"], got["g"] - gu), 0.0)
    rn = n1.cpu().numpy()
    assert rn[0] == viol.max()
    assert abs(rn[1] - (viol ** 2).sum()) <= 1e-12 * (viol ** 2).sum()
    sep = prob.residual_norms(out["g"]).cpu().numpy()
    assert sep[0] == rn[0]


def test_fused_residual_norms_empty_batch():
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import make_problem

    prob = make_problem(4, "ground")
    dev = torch.device("cuda:0")
    xt = torch.empty(0, prob.n, dtype=torch.float64, device=dev)
    out = prob.eval_batch(xt, outputs=("g", "norms"), out={"norms": torch.full((2,), 7.0, dtype=torch.float64, device=dev)})
    assert out["norms"].cpu().tolist() == [0.0, 0.0]
    with pytest.raises(_abi.InvalidArgument):
        prob.eval_batch(torch.zeros(3, prob.n, dtype=torch.float64, device=dev), outputs=("jac", "norms"))


@pytest.mark.parametrize("N", [4, 16])
@pytest.mark.parametrize("pattern", ["all_sq", "all_ground", "sparse_sq", "alternating", "blocks"])
def test_mixed_tag_patterns_layouts(N, pattern):
    """Mixed batches with every tag pattern (homogeneous, sparse, alternating, blocks straddling
    tiles): every output equals the oracle, and the values-only and entry-major layouts equal the
    IFOPT layout bit for bit (the tile kernel compacts each tile's instances by kind)."""
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, "mixed")
    B = 1000
    x, mass, _ = generate(N, "mixed", B, 77 + N)
    i = np.arange(B)
    tag = {"all_sq": np.full(B, 2), "all_ground": np.full(B, 1), "sparse_sq": np.where(i % 10 == 3, 2, 1),
           "alternating": np.where(i % 2 == 0, 2, 1), "blocks": np.where((i // 37) % 3 == 0, 2, 1)}[pattern]
    tag = tag.astype(np.uint8)
    got, ref = _run(prob, x, mass, tag)
    _check(prob, "mixed", x, got, ref, tag)
    dev = torch.device("cuda:0")
    xt, mt, tt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev), torch.tensor(tag, device=dev)
    soa = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "grad"), soa=True)
    torch.cuda.synchronize()
    for k in ("g", "jac", "grad"):
        assert np.array_equal(soa[k].cpu().numpy().T, got[k], equal_nan=True), k
    folded = prob.eval_batch(xt, mt, tt, outputs=("g", "jac"), jac_folded=True)
    torch.cuda.synchronize()
    var_k = prob.jac_fold_info()[0]
    assert np.array_equal(folded["jac"].cpu().numpy(), got["jac"][:, var_k], equal_nan=True)
    assert np.array_equal(folded["g"].cpu().numpy(), got["g"], equal_nan=True)
