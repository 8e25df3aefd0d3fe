"""Values-only ("folded") Jacobian records and entry-major (SoA) outputs of cpl_eval_batch_ex.

The folded layout skips the entries that are the same for every x:
the force-balance I3 blocks (src/Constraints/CentroidalStatics.cpp:93-95), the normal rows' n_r
ones (src/Constraints/EnvironmentNormal.cpp:63-70) and, on Ground, the gradient (0, 0, 1)
(src/Ground.cpp:30-35) and the zero normal Jacobian (src/Ground.cpp:46-50).
CPU: the layout partitions the CSR positions and the constants are what the oracle writes there at
any x.  GPU: folded values scattered back with the constants == cpl_eval_batch's CSR values, bit for
bit (NaN positions included), on every kernel variant; SoA == the transposed instance-major outputs.
"""
import numpy as np
import pytest

import pyoracle

torch = pytest.importorskip("torch")

CASES = [("ground", 1), ("ground", 4), ("ground", 12), ("superquadric", 4), ("superquadric", 8), ("mixed", 16),
         ("none", 4), ("none", 3)]


@pytest.mark.parametrize("env,N", CASES)
def test_fold_info_partitions_structure_and_constants_match_oracle(env, N):
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    n, m, nnz = prob.get_nlp_info()
    var_k, const_k, const_val = prob.jac_fold_info()
    per_contact = {"ground": 12, "none": 12}.get(env, 24)
    assert var_k.size == 6 + 12 * N + per_contact * N
    assert var_k.size + const_k.size == nnz
    assert np.array_equal(np.sort(np.concatenate([var_k, const_k])), np.arange(nnz))
    assert (np.diff(var_k) > 0).all() and (np.diff(const_k) > 0).all()
    if env == "ground":
        assert const_k.size == 18 * N          # 72 of 174 at N = 4: 1952 -> 1376 B per instance
    x, mass, tag = generate(N, env, 97, 5 + N)
    x[0] = 0.0                                  # IPOPT's start point: 0/0 cone entries are not constants
    ref = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=("jac",))["jac"]
    assert np.array_equal(ref[:, const_k], np.broadcast_to(const_val, (x.shape[0], const_k.size)))


def test_fold_info_rejects_bad_desc():
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import make_problem

    d = make_problem(4, "ground").desc()
    d.n_contacts = 0
    with pytest.raises(_abi.CplError):
        _abi.check(_abi.lib.cpl_jac_fold_info(d, None, None, None, None, None))


def _scatter(prob, folded):
    _, _, nnz = prob.get_nlp_info()
    var_k, const_k, const_val = prob.jac_fold_info()
    full = np.empty((folded.shape[0], nnz))
    full[:, var_k] = folded
    full[:, const_k] = const_val
    return full


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("env,N", CASES)
def test_folded_equals_csr_bitwise(variant, env, N):
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    B = 1031
    x, mass, tag = generate(N, env, B, 61 + N)
    x[::97] = 0.0                               # NaN entries (0/0 cones) keep their positions
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
    try:
        full = prob.eval_batch(xt, mt, tt, outputs=("g", "jac"))
        fo = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"), jac_folded=True)
        torch.cuda.synchronize()
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    J = full["jac"].cpu().numpy()
    assert np.array_equal(_scatter(prob, fo["jac"].cpu().numpy()), J, equal_nan=True)
    assert torch.equal(fo["g"], full["g"]) or np.array_equal(fo["g"].cpu().numpy(), full["g"].cpu().numpy(),
                                                              equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 2, 3])
@pytest.mark.parametrize("env,N", [("ground", 4), ("superquadric", 8), ("mixed", 16), ("none", 3)])
@pytest.mark.parametrize("folded", [False, True])
def test_soa_is_transposed_aos(variant, env, N, folded):
    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(N, env)
    B = 777
    x, mass, tag = generate(N, env, B, 7 + N)
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    outs = ("g", "jac", "f", "grad", "norms")
    _abi.check(_abi.lib.cpl_set_tuning(variant, 0, 256, 1, 0))
    try:
        aos = prob.eval_batch(xt, mt, tt, outputs=outs, jac_folded=folded)
        soa = prob.eval_batch(xt, mt, tt, outputs=outs, jac_folded=folded, soa=True)
        torch.cuda.synchronize()
    finally:
        _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    for k in ("g", "jac", "grad"):
        assert soa[k].shape == (aos[k].shape[1], B)
        assert torch.equal(soa[k], aos[k].t())
    assert torch.equal(soa["f"], aos["f"])
    # [max violation, sum of squares]: the max exactly; the sum is summed per kernel tile, and by default
    # a mixed AoS batch runs the kind split (two kernels' partials) where the SoA one runs the interleaved
    # kernel — the same terms in another order, equal to rounding
    assert soa["norms"][0] == aos["norms"][0]
    assert float(soa["norms"][1]) == pytest.approx(float(aos["norms"][1]), rel=1e-12, abs=1e-300)


@pytest.mark.gpu
def test_folded_north_star_bytes():
    """1,048,576 x 4 Ground in the folded layout: 1376 B per instance, the same values."""
    from centroidalplanner_amd.workload import CONFIGS, config_inputs

    prob, x, mass, _ = config_inputs(CONFIGS["ground4_1m"])
    dev = torch.device("cuda:0")
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    fo = prob.eval_batch(xt, mt, outputs=("g", "jac"), jac_folded=True)
    assert fo["jac"].shape == (x.shape[0], 102)
    assert 8 * (prob.n + 1 + prob.m + fo["jac"].shape[1]) == 1376
    var_k, _, _ = prob.jac_fold_info()
    full = prob.eval_batch(xt, mt, outputs=("jac",))["jac"]
    assert torch.equal(full[:, torch.as_tensor(var_k.astype(np.int64), device=dev)], fo["jac"])
