"""The batched solve loop (centroidalplanner_amd/batch_ipm.py, BASELINE.json configs[4]).

CPU: the solver's host logic driven by the oracle's callbacks (test infrastructure), on a few
instances of the TestBasic ground scenario (tests/TestBasic.cpp:64-135) with the reference's
default force weight; every solution is certified independently:
  * TestBasic's own assertions (force / torque balance with the manipulation wrench, contacts on
    the ground, unit normals, friction cones, bounds);
  * a first-order KKT certificate of the returned primal-dual pair through the oracle's callbacks
    (stationarity, sign and complementarity of the cone multipliers);
  * the objective is at least as good as an independent single-instance solve (SLSQP over the same
    callbacks; the problem is nonconvex, so both are local optima).
GPU: the same solve with the product callbacks (the HIP kernel through cpl_eval_batch) on a larger
batch, checked with the same certificates and against the oracle-driven batched solve.
"""
import numpy as np
import pytest

import pyoracle
from centroidalplanner_amd.batch_ipm import STATUS_ACCEPTABLE, batch_ipm_solve
from centroidalplanner_amd.workload import MU, GROUND_Z, WRENCH, solve_inputs, solve_problem

torch = pytest.importorskip("torch")


class OracleBatchEvaluator:
    """Batched callbacks through the CPU restatement, on CPU torch tensors; `hessian` is the oracle's
    restatement of the analytic Lagrangian Hessian (Ground / no environment; None otherwise, and the
    solve loop differences the Lagrangian gradient instead)."""

    def __init__(self, problem, nthreads=4):
        self.problem = problem
        self.nthreads = nthreads

    def __call__(self, X, mass, outputs=("g", "jac", "f", "grad")):
        o = pyoracle.eval_batch(self.problem.desc(), X.cpu().numpy(), None if mass is None else mass.cpu().numpy(),
                                None, outputs=tuple(outputs), nthreads=self.nthreads)
        return {k: torch.as_tensor(v, device=X.device) for k, v in o.items()}

    def hessian(self, X, y, free, zero_cost=False):
        """zero_cost: the Hessian of y^T g alone (the template with zero cost weights — the
        restoration phase's constraint curvature)."""
        if self.problem.desc().env_kind not in (0, 1):
            return None
        d = self.problem.desc()
        if zero_cost:
            d = type(d).from_buffer_copy(d)
            d.W_com = 0.0
            for i in range(len(d.W_F)):
                d.W_F[i] = 0.0
                d.W_p[i] = 0.0
        H = pyoracle.lagrangian_hessian(d, X.cpu().numpy(), y.cpu().numpy(), free.cpu().numpy())
        return torch.as_tensor(H, device=X.device)


def _certify(prob, x, y, mass, tol_kkt=1e-7):
    """TestBasic.cpp:101-132 assertions + a KKT certificate through the oracle at x."""
    n, m, _ = prob.get_nlp_info()
    xl, xu, gl, gu = prob.get_bounds_info()
    N = len(prob.contact_names)
    c = x[0:3]
    F_sum, T_sum = np.zeros(3), np.zeros(3)
    for i in range(N):
        F, p, nv = x[3 + 9 * i: 6 + 9 * i], x[6 + 9 * i: 9 + 9 * i], x[9 + 9 * i: 12 + 9 * i]
        F_sum += F
        T_sum += np.cross(p - c, F)
        assert p[2] == pytest.approx(GROUND_Z, abs=1e-6)
        assert np.linalg.norm(nv) == pytest.approx(1.0, abs=1e-6)
        assert nv[2] == pytest.approx(1.0, abs=1e-6)
        assert -F.dot(nv) <= 1e-9
        assert np.linalg.norm(F - nv.dot(F) * nv) - MU * F.dot(nv) <= 1e-7
    assert F_sum[0] == pytest.approx(WRENCH[0], abs=1e-6)
    assert F_sum[1] == pytest.approx(WRENCH[1], abs=1e-6)
    assert F_sum[2] == pytest.approx(mass * 9.81 + WRENCH[2], abs=1e-6)
    np.testing.assert_allclose(T_sum, WRENCH[3:], atol=1e-5)
    assert (x >= xl - 1e-9).all() and (x <= xu + 1e-9).all()
    # first-order certificate of the returned primal-dual pair, through the oracle's callbacks:
    # stationarity grad f + J^T y = 0 (bounds inactive), y >= 0 on the cone rows (g <= 0) and
    # complementarity y_r g_r = 0 there
    o = pyoracle.eval_batch(prob.desc(), x[None], np.array([mass]), None, outputs=("g", "jac", "f", "grad"))
    iR, jC = prob.get_structure()
    J = np.zeros((m, n))
    J[iR, jC] = np.nan_to_num(o["jac"][0])
    g = o["g"][0]
    res = o["grad"][0] + J.T @ y
    bound_act = (np.abs(x - xl) <= 1e-6) | (np.abs(x - xu) <= 1e-6)
    res[bound_act] = 0.0
    scale = max(1.0, np.abs(o["grad"][0]).max())
    assert np.abs(res).max() <= tol_kkt * scale
    ineq = gl != gu
    ymax = max(1.0, np.abs(y).max())
    assert (y[ineq] >= -1e-8 * ymax).all()
    assert (np.abs(y[ineq] * g[ineq]) <= 1e-6 * ymax).all()
    return float(o["f"][0])


def _slsqp_objective(prob, x0, mass):
    from slsqp_ref import slsqp_solve

    class E:
        def eval_batch(self, X):
            X = np.atleast_2d(X)
            return pyoracle.eval_batch(prob.desc(), X, np.full(X.shape[0], mass), None,
                                       outputs=("g", "jac", "f", "grad"), nthreads=1)

    r = slsqp_solve(prob, E(), x0=x0, tol=1e-12, max_iter=500)
    o = E().eval_batch(r.x)
    return float(o["f"][0])


def test_batch_solve_oracle_cpu():
    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    X0, mass = solve_inputs(prob, 6, seed=11)
    r = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob),
                        max_iter=200)
    assert bool((r.status <= STATUS_ACCEPTABLE).all()), r.status
    assert r.iterations_run < 100
    for b in range(X0.shape[0]):
        x = r.x[b].numpy()
        f = _certify(prob, x, r.y[b].numpy(), mass[b])
        assert f == pytest.approx(float(r.objective[b]), rel=1e-12)
        if b < 3:
            # the problem is nonconvex (bilinear torque balance): both points are certified local
            # optima.  Instances 0 and 1 reach SLSQP's optimum or a better one (0: 2.2 % below, 1: equal);
            # with IPOPT's gradient-based scaling the interior-point path of instance 2 ends in the
            # neighbouring optimum 0.53 % above SLSQP's (unscaled it had reached SLSQP's), pinned here
            # on its own so that a regression of 0 or 1 cannot hide under its tolerance
            ref = _slsqp_objective(prob, X0[b], mass[b])
            if b < 2:
                assert f <= ref * (1.0 + 1e-7)
            else:
                assert f == pytest.approx(188518.53629546892, rel=1e-8)
                assert f <= ref * (1.0 + 6e-3)


def test_batch_solve_rejects_host_inputs_without_gpu_callbacks():
    """The product evaluator is the HIP kernel: host tensors are refused, never evaluated on the CPU."""
    from centroidalplanner_amd._abi import CplError

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    X0, mass = solve_inputs(prob, 2)
    with pytest.raises(CplError):
        batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), max_iter=2)


@pytest.mark.gpu
def test_batch_solve_gpu_kernel_callbacks():
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    B = 512
    X0, mass = solve_inputs(prob, B, seed=5)
    dev = torch.device("cuda:0")
    ev = KernelEvaluator(prob)
    r = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), evaluator=ev,
                        max_iter=200)
    assert r.graph and ev.calls >= 3  # the iteration was captured with the kernel callbacks in it
    st = r.status.cpu().numpy()
    assert (st <= STATUS_ACCEPTABLE).all()
    X = r.x.cpu().numpy()
    Y = r.y.cpu().numpy()
    obj = r.objective.cpu().numpy()
    # certify a sample; compare a smaller sample with the oracle-driven batched solve (same algorithm)
    for b in range(0, B, 37):
        f = _certify(prob, X[b], Y[b], mass[b])
        assert f == pytest.approx(obj[b], rel=1e-12)
    sub = np.arange(0, B, 64)
    rc = batch_ipm_solve(prob, torch.as_tensor(X0[sub]), torch.as_tensor(mass[sub]),
                         evaluator=OracleBatchEvaluator(prob), max_iter=200)
    np.testing.assert_allclose(obj[sub], rc.objective.numpy(), rtol=1e-8)


# ---- the other TestBasic scenarios, many instances at once (per-instance robot masses) -------------
def _scenario(which):
    """TestBasic.cpp:138-222 (Superquadric, force weight 0 as in the test) and :225-292 (CoMPlanner:
    fixed contact positions / normals, contact4 lifting, thresholds 20)."""
    from centroidalplanner_amd import CentroidalPlanner, CoMPlanner, Superquadric

    names = ["contact1", "contact2", "contact3", "contact4"]
    if which == "superquadric":
        env = Superquadric()
        env.SetMu(MU)
        env.SetParameters([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [10.0, 10.0, 10.0])
        cpl = CentroidalPlanner(names, 100.0, env)
        cpl.SetForceWeight(0.0)
        for c in names:
            cpl.SetPosBounds(c, np.array([-0.5, -0.5, 0.5]), np.array([0.5, 0.5, 1.5]))
        cpl.SetManipulationWrench(WRENCH)
        prob = cpl.GetCplProblem()
        x0 = np.zeros(prob.n)
        x0[0:3] = [0.0, 0.0, 1.0]
        for i, (px, py) in enumerate([(0.3, 0.0), (0.0, 0.3), (-0.3, 0.0), (0.0, -0.3)]):
            nrm = -np.array([px, py, 0.0]) / 0.3
            x0[3 + 9 * i: 6 + 9 * i] = nrm * 300.0 + np.array([0.0, 0.0, 250.0])
            x0[6 + 9 * i: 9 + 9 * i] = [px, py, 1.0 + 0.01 * (i - 1.5)]
            x0[9 + 9 * i: 12 + 9 * i] = nrm
        wrench = WRENCH
    else:
        cpl = CoMPlanner(names, 100.0)
        cpl.SetMu(MU)
        for c, p in zip(names, ([1.0, 1.0, 0.0], [-1.0, 1.0, 0.0], [-1.0, -1.0, 0.0], [1.0, -1.0, 0.0])):
            cpl.SetContactPosition(c, p)
        cpl.SetLiftingContact("contact4")
        for c in names:
            cpl.SetForceThreshold(c, 20.0)
        prob = cpl.GetCplProblem()
        x0 = np.zeros(prob.n)
        x0[0:3] = [0.0, 0.0, 1.0]
        for i in range(4):
            x0[3 + 9 * i: 6 + 9 * i] = [1.0, 1.0, 330.0]
        wrench = np.zeros(6)
    xl, xu, _, _ = prob.get_bounds_info()
    return prob, np.clip(x0, xl, xu), wrench


def _certify_scenario(which, prob, x, mass, wrench):
    """TestBasic's own assertions for the scenario (TestBasic.cpp:187-220 / :271-290)."""
    C, R, P = np.array([0.0, 0.0, 1.0]), np.array([0.3, 0.3, 10.0]), np.array([10.0, 10.0, 10.0])
    xl, xu, _, _ = prob.get_bounds_info()
    assert (x >= xl).all() and (x <= xu).all()
    c = x[0:3]
    F_sum, T_sum = np.zeros(3), np.zeros(3)
    for i in range(4):
        F, p, nv = x[3 + 9 * i: 6 + 9 * i], x[6 + 9 * i: 9 + 9 * i], x[9 + 9 * i: 12 + 9 * i]
        F_sum += F
        T_sum += np.cross(p - c, F)
        assert -F.dot(nv) <= 1e-9
        assert np.linalg.norm(F - nv.dot(F) * nv) - MU * F.dot(nv) <= 1e-7
        if which == "superquadric":
            assert sum(((p[k] - C[k]) / R[k]) ** P[k] for k in range(3)) == pytest.approx(1.0, abs=1e-4)
            assert np.linalg.norm(nv) == pytest.approx(1.0, abs=1e-6)
    assert F_sum[0] == pytest.approx(wrench[0], abs=1e-6)
    assert F_sum[1] == pytest.approx(wrench[1], abs=1e-6)
    assert F_sum[2] == pytest.approx(mass * 9.81 + wrench[2], abs=1e-6)
    np.testing.assert_allclose(T_sum, wrench[3:], atol=1e-4)
    if which == "com":  # the lifting contact carries no force
        np.testing.assert_array_equal(x[3 + 27: 6 + 27], 0.0)


# the Hessian mode per scenario: IPOPT's exact Hessian on the exponent-10 superquadric surface (the
# limited-memory model stalls there), IFOPT's limited-memory model on CoMPlanner (whose held contact
# sits on the cone's kink at zero tangential force, where the exact Hessian of |F_t| is unbounded)
_HESSIAN = {"superquadric": "exact", "com": "limited-memory"}


@pytest.mark.parametrize("which", ["superquadric", "com"])
def test_batch_solve_other_scenarios_oracle_cpu(which):
    prob, x0, wrench = _scenario(which)
    B = 4
    mass = np.random.default_rng(3).uniform(80.0, 150.0, B)
    r = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1))), torch.as_tensor(mass),
                        evaluator=OracleBatchEvaluator(prob), max_iter=300, hessian=_HESSIAN[which])
    assert bool((r.status <= STATUS_ACCEPTABLE).all()), r.status
    for b in range(B):
        _certify_scenario(which, prob, r.x[b].numpy(), mass[b], wrench)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["superquadric", "com"])
def test_batch_solve_other_scenarios_gpu(which):
    prob, x0, wrench = _scenario(which)
    B = 256
    mass = np.random.default_rng(4).uniform(80.0, 150.0, B)
    dev = torch.device("cuda:0")
    r = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1)), device=dev), torch.as_tensor(mass, device=dev),
                        max_iter=1000, hessian=_HESSIAN[which])
    assert r.graph
    st = r.status.cpu().numpy()
    ok = st <= STATUS_ACCEPTABLE
    assert ok.all(), np.bincount(st)
    X = r.x.cpu().numpy()
    for b in np.flatnonzero(ok)[::17]:
        _certify_scenario(which, prob, X[b], mass[b], wrench)


@pytest.mark.gpu
def test_fused_lagrangian_grad_is_bitwise_the_two_launch_result():
    """cpl_eval_lagrangian_grad (grad f + J^T y from the eval kernel's LDS tile) against
    cpl_eval_batch (jac, grad) + cpl_lagrangian_grad: the same operations in the same order."""
    import ctypes

    from centroidalplanner_amd import _abi
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    n, m, nnz = prob.get_nlp_info()
    X0, mass = solve_inputs(prob, 333, seed=5)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(6)
    X = torch.as_tensor(X0 + rng.normal(scale=0.05, size=X0.shape), device=dev).contiguous()
    X[::7, 3:5] = 0.0  # zero tangential force on a contact: the 0/0 cone Jacobian entries (NaN -> 0)
    M = torch.as_tensor(mass, device=dev)
    rep = 3
    y = torch.as_tensor(rng.normal(size=((X.shape[0] + rep - 1) // rep, m)), device=dev).contiguous()
    iRow, jCol = prob.get_structure()
    order = np.lexsort((iRow, jCol))
    col_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(col_ptr, jCol.astype(np.int64) + 1, 1)
    col_ptr = np.cumsum(col_ptr)
    csc = [torch.as_tensor(a.astype(np.int32), device=dev) for a in (col_ptr, order, iRow[order])]
    fused = KernelEvaluator(prob).lagrangian_grad(X, M, y, rep, csc)
    assert fused is not None
    o = prob.eval_batch(X, M, outputs=("jac", "grad"))
    ref = torch.empty_like(fused)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _abi.check(_abi.lib.cpl_lagrangian_grad(X.shape[0], n, m, nnz, p(csc[0]), p(csc[1]), p(csc[2]), p(o["grad"]),
                                            p(o["jac"]), p(y), rep, p(ref), None))
    torch.cuda.synchronize()
    assert torch.isfinite(ref).all()
    assert torch.equal(fused, ref)
    # converged instances skipped: the active ones bitwise the same, the others untouched
    active = torch.as_tensor(rng.uniform(size=y.shape[0]) < 0.5, device=dev)
    masked = KernelEvaluator(prob).lagrangian_grad(X, M, y, rep, csc, active)
    torch.cuda.synchronize()
    rows = active.repeat_interleave(rep)[: X.shape[0]]
    assert torch.equal(masked[rows], ref[rows])


@pytest.mark.gpu
def test_batch_solve_gpu_eight_contacts():
    """The loop at N = 8 (configs[2]'s contact count on Ground: nw = 91, m = 54 — a 119 KiB KKT LDS
    image), every instance certified like the 4-contact case."""
    cpl = solve_problem(n_contacts=8)
    prob = cpl.GetCplProblem()
    B = 128
    X0, mass = solve_inputs(prob, B, seed=8)
    dev = torch.device("cuda:0")
    r = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), max_iter=300)
    assert r.graph
    st = r.status.cpu().numpy()
    assert (st <= STATUS_ACCEPTABLE).all(), np.bincount(st)
    X, Y = r.x.cpu().numpy(), r.y.cpu().numpy()
    for b in range(0, B, 16):
        _certify(prob, X[b], Y[b], mass[b])


def test_batch_solve_limited_memory_oracle_cpu():
    """IFOPT's default Hessian mode (the reference's IpoptSolver keeps it: src/CentroidalPlanner.cpp:22-29):
    IPOPT's limited-memory BFGS model (6 pairs, scalar1), on the host path over the oracle's callbacks."""
    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    X0, mass = solve_inputs(prob, 4, seed=11)
    r = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob),
                        max_iter=1000, hessian="limited-memory")
    assert bool((r.status <= STATUS_ACCEPTABLE).all()), r.status
    for b in range(X0.shape[0]):
        _certify(prob, r.x[b].numpy(), r.y[b].numpy(), mass[b], tol_kkt=1e-5)


@pytest.mark.gpu
def test_batch_solve_gpu_limited_memory():
    """The limited-memory (L-BFGS) mode on the device with the kernel callbacks, graph-captured."""
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    B = 256
    X0, mass = solve_inputs(prob, B, seed=9)
    dev = torch.device("cuda:0")
    ev = KernelEvaluator(prob)
    r = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), evaluator=ev,
                        max_iter=1000, hessian="limited-memory")
    assert r.graph
    st = r.status.cpu().numpy()
    assert (st <= STATUS_ACCEPTABLE).all(), np.bincount(st)
    X, Y = r.x.cpu().numpy(), r.y.cpu().numpy()
    for b in range(0, B, 23):
        _certify(prob, X[b], Y[b], mass[b], tol_kkt=1e-5)
    sub = np.arange(0, B, 64)
    rc = batch_ipm_solve(prob, torch.as_tensor(X0[sub]), torch.as_tensor(mass[sub]), evaluator=OracleBatchEvaluator(prob),
                         max_iter=1000, hessian="limited-memory")
    np.testing.assert_allclose(r.objective.cpu().numpy()[sub], rc.objective.numpy(), rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("hessian", ["exact", "limited-memory"])
def test_active_set_compaction_is_exact(hessian):
    """The native engine's active-set compaction (the lock-step batch shrinks to its active
    instances) leaves every instance's iterates untouched: the same x, y, status and iteration
    counts, bit for bit, as the solve that keeps every row to the end."""
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    B = 1024
    X0, mass = solve_inputs(prob, B, seed=13)
    dev = torch.device("cuda:0")
    X0t, mt = torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev)
    a = batch_ipm_solve(prob, X0t, mt, evaluator=KernelEvaluator(prob), max_iter=1000, hessian=hessian, compact=True)
    b = batch_ipm_solve(prob, X0t, mt, evaluator=KernelEvaluator(prob), max_iter=1000, hessian=hessian, compact=False)
    assert a.compactions >= 1 and b.compactions == 0
    for k in ("x", "y", "status", "iterations", "objective", "primal_inf", "dual_inf"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


@pytest.mark.gpu
@pytest.mark.parametrize("max_ls,max_soc,hessian", [(4, 1, "limited-memory"), (4, 0, "exact"), (1, 1, "exact"),
                                                    (2, 2, "limited-memory")])
def test_split_small_batch_iterations_are_exact(max_ls, max_soc, hessian):
    """Small batches run each iteration as three graphs and skip the later line-search trials and the
    feasibility step when nothing is still searching after the first trial (its second-order
    correction fused with the halving and the any-searching flag): bitwise the eager one-step
    iteration, for every line-search / SOC configuration."""
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    cpl = solve_problem()
    prob = cpl.GetCplProblem()
    B = 32
    X0, mass = solve_inputs(prob, B, seed=21)
    dev = torch.device("cuda:0")
    X0t, mt = torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev)
    kw = dict(max_iter=1000, hessian=hessian, max_ls=max_ls, max_soc=max_soc)
    a = batch_ipm_solve(prob, X0t, mt, evaluator=KernelEvaluator(prob), graph=True, **kw)
    b = batch_ipm_solve(prob, X0t, mt, evaluator=KernelEvaluator(prob), graph=False, **kw)
    assert a.graph and not b.graph
    for k in ("x", "y", "status", "iterations", "objective"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    if max_ls == 1:  # one trial per iteration, no backtracking (a stress setting, not IPOPT's): on the scaled
        # problem (nlp_scaling, round 5) one instance of the 32 cycles to the iteration limit: at most that one
        assert int((a.status > STATUS_ACCEPTABLE).sum()) <= 1
    else:
        assert bool((a.status <= STATUS_ACCEPTABLE).all())


@pytest.mark.gpu
@pytest.mark.parametrize("nlp_scaling", ["gradient-based", "none"])
def test_device_nlp_scaling_matches_host(nlp_scaling):
    """The engine's NLP scaling (cpl_solve_options.nlp_scaling) against the host restatement over the
    oracle's callbacks, scaling on and off: the same outcomes and iteration counts, objectives to
    1e-8, and the returned multipliers (unscaled: dc y / df) certify the unscaled problem's KKT point."""
    from centroidalplanner_amd.batch_ipm import KernelEvaluator

    prob = solve_problem().GetCplProblem()
    B = 8
    X0, mass = solve_inputs(prob, B, seed=17)
    dev = torch.device("cuda:0")
    r = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev),
                        evaluator=KernelEvaluator(prob), max_iter=300, hessian="exact", nlp_scaling=nlp_scaling)
    h = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob),
                        max_iter=300, hessian="exact", nlp_scaling=nlp_scaling)
    assert torch.equal(r.status.cpu(), h.status) and bool((h.status == 0).all())
    assert torch.equal(r.iterations.cpu(), h.iterations)
    np.testing.assert_allclose(r.objective.cpu().numpy(), h.objective.numpy(), rtol=1e-8)
    X, Y = r.x.cpu().numpy(), r.y.cpu().numpy()
    for b in range(B):
        _certify(prob, X[b], Y[b], mass[b])
