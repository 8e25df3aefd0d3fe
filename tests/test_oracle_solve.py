"""The compiled solve restatement (oracle/cpl_solve_host.c — the CPU baseline of bench.py's solve
legs) against the host path of the batched solver (batch_ipm.py over the oracle's callbacks): the
same iteration, so the same status, iteration count and restoration count, and the same point and
objective to rounding (the dense factorisations differ in summation order).  IPOPT itself is not in
the image; both restate its method (parity of the method: test_oracle_pinning.py)."""
import warnings

import numpy as np
import pytest

import pyoracle
from centroidalplanner_amd.batch_ipm import batch_ipm_solve
from centroidalplanner_amd.workload import solve_inputs, solve_problem
from test_batch_solve import OracleBatchEvaluator

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("hessian,max_iter", [("limited-memory", 1000), ("exact", 300)])
def test_compiled_solve_matches_host_path(hessian, max_iter):
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 3)
    for b in range(3):
        c = pyoracle.solve(prob.desc(), X0[b], mass[b], max_iter=max_iter, hessian=hessian)
        h = batch_ipm_solve(prob, torch.as_tensor(X0[b:b + 1]), torch.as_tensor(mass[b:b + 1]), max_iter=max_iter,
                            evaluator=OracleBatchEvaluator(prob, 1), hessian=hessian)
        assert c["status"] == int(h.status[0]) == 0
        assert c["iterations"] == int(h.iterations[0])
        assert c["restorations"] == int(h.restorations[0])
        np.testing.assert_allclose(c["x"], h.x[0].numpy(), rtol=0, atol=1e-9)
        assert c["objective"] == pytest.approx(float(h.objective[0]), rel=1e-12)


def test_compiled_solve_from_zero_simple_problem():
    """TestBasic.cpp:28-61 (one contact, Ground z = 0.1) from x = 0 under IFOPT's defaults: the same
    outcome as the host path (test_oracle_pinning.test_simple_problem's assertions)."""
    from centroidalplanner_amd import CentroidalPlanner, Ground

    env = Ground()
    env.SetGroundZ(0.1)
    prob = CentroidalPlanner(["contact1"], 100.0, env).GetCplProblem()
    x0 = prob.get_starting_point()
    c = pyoracle.solve(prob.desc(), x0, 100.0)
    h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), None, evaluator=OracleBatchEvaluator(prob, 1),
                        hessian="limited-memory")
    assert c["status"] <= 1 and c["status"] == int(h.status[0])
    assert c["iterations"] == int(h.iterations[0])
    x = c["x"]
    assert x[8] == pytest.approx(0.1, abs=1e-6)          # contact z on the ground
    assert x[5] == pytest.approx(981.0, abs=1e-6)        # vertical force carries m g
    assert x[11] == pytest.approx(1.0, abs=1e-6)         # normal (0, 0, 1)


def test_time_solve_reports_per_instance_outcomes():
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 4)
    t, st, it = pyoracle.time_solve(prob.desc(), X0, mass, max_iter=1000)
    assert t > 0 and st.shape == (4,) and (st == 0).all() and (it > 0).all()


@pytest.mark.parametrize("hessian", ["limited-memory", "exact"])
def test_nlp_scaling_off_switch_and_effect(hessian):
    """IPOPT's gradient-based scaling is active on the solve workload (its torque rows' gradients reach
    ~1.3e3 at the start, the cone rows ~3e2): the compiled and the host restatement agree with it off
    (nlp_scaling "none" on both) as with it on, and switching it changes the trajectory."""
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 2)
    for b in range(2):
        pyoracle.set_nlp_scaling("none")
        try:
            c0 = pyoracle.solve(prob.desc(), X0[b], mass[b], max_iter=1000, hessian=hessian)
        finally:
            pyoracle.set_nlp_scaling("gradient-based")
        h0 = batch_ipm_solve(prob, torch.as_tensor(X0[b:b + 1]), torch.as_tensor(mass[b:b + 1]), max_iter=1000,
                             evaluator=OracleBatchEvaluator(prob, 1), hessian=hessian, nlp_scaling="none")
        assert c0["status"] == int(h0.status[0]) == 0
        assert c0["iterations"] == int(h0.iterations[0])
        np.testing.assert_allclose(c0["x"], h0.x[0].numpy(), rtol=0, atol=1e-9)
        c1 = pyoracle.solve(prob.desc(), X0[b], mass[b], max_iter=1000, hessian=hessian)
        assert c1["status"] == 0
        assert c1["iterations"] != c0["iterations"] or np.abs(c1["x"] - c0["x"]).max() > 1e-12


# ---- where the two restatements part (round 6; DESIGN.md section 5, "The CPU baseline's iteration") ----
@pytest.mark.parametrize("hessian,min_equal_iters,max_absdiff", [("exact", 1.0, 0), ("limited-memory", 0.75, 10)])
def test_compiled_vs_host_solve5_sample(hessian, min_equal_iters, max_absdiff):
    """256 instances of the solve workload: the compiled restatement (the solve legs' CPU baseline) and
    the host restatement reach the same status on every instance.  Exact Hessian: the same iteration
    count on every instance (measured 256/256).  IPOPT's L-BFGS: the dense model's recursion is summed in
    different orders (C loops against torch's batched products), and on the scaled problem those
    last-bit differences move the line search's acceptance by a trial now and then: stated bound
    >= 75 % equal iteration counts and no instance more than 10 apart (measured 83 %, at most 7)."""
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 256)
    _, st, it = pyoracle.time_solve(prob.desc(), X0, mass, max_iter=3000, hessian=hessian)
    h = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob, 4),
                        hessian=hessian, max_iter=3000)
    hs, hi = h.status.numpy(), h.iterations.numpy()
    assert (hs == st).all() and (st <= 1).all()
    assert float((hi == it).mean()) >= min_equal_iters
    assert int(np.abs(hi.astype(np.int64) - it).max()) <= max_absdiff


def _testbasic(name):
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import testbasic_outcomes as tb

    make = {"testSimpleProblem": tb.simple, "testGroundEnv": tb.ground, "testSuperquadricEnv": tb.superquadric,
            "testCoMPlanner": tb.com_planner}[name]
    cpl, wrench, mu = make()
    prob = cpl.GetCplProblem()
    xl, xu, _, _ = prob.get_bounds_info()
    return prob, np.clip(prob.get_starting_point(), xl, xu), float(prob.desc().mass)


def _jacobian_w(prob, x, mass):
    """A = [J_free | -P] (NaN as 0, the solvers' policy) at x."""
    n, m, _ = prob.get_nlp_info()
    xl, xu, gl, gu = prob.get_bounds_info()
    o = pyoracle.eval_batch(prob.desc(), x[None], np.array([mass]), None, outputs=("g", "jac"))
    iR, jC = prob.get_structure()
    J = np.zeros((m, n))
    J[iR, jC] = np.nan_to_num(o["jac"][0])
    free = xl != xu
    ineq = np.nonzero(gl != gu)[0]
    P = np.zeros((m, len(ineq)))
    P[ineq, np.arange(len(ineq))] = 1.0
    return np.hstack([J[:, free], -P])


@pytest.mark.parametrize("name", ["testGroundEnv", "testSuperquadricEnv"])
def test_testbasic_rank_deficient_start_parts_the_restatements(name):
    """TestBasic's x = 0 starts of the ground and Superquadric scenarios: every force is 0, so the torque
    rows' CoM columns and FrictionCone's rows (0/0, taken as 0) vanish and A is rank deficient — the
    first Newton step is 1e9-sized along a direction set by rounding (delta_c is added to R's pivots
    with their noisy signs), so the two restatements' FIRST iterates already differ.  Both still end at
    points that meet TestBasic's assertions (test_oracle_pinning.py for the host path and the GPU)."""
    prob, x0, mass = _testbasic(name)
    s = np.linalg.svd(_jacobian_w(prob, x0, mass), compute_uv=False)
    assert s[-1] <= 1e-12 * s[0]  # numerically rank deficient at the start
    c = pyoracle.solve(prob.desc(), x0, mass, max_iter=1)
    h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), max_iter=1,
                        evaluator=OracleBatchEvaluator(prob, 1), hessian="limited-memory")
    assert np.abs(c["x"] - h.x[0].numpy()).max() > 1e-6  # the documented divergence at the first iterate


def test_testbasic_com_planner_parts_at_the_cone_kink():
    """TestBasic's CoMPlanner scenario from x = 0: the first iterates agree to rounding; there the
    contacts' tangential forces are rounding residue (|F_t| ~ 1e-31 against F_n ~ 0.24), and
    FrictionCone's row-1 Jacobian (src/Constraints/FrictionCone.cpp:85-99) takes F_t / |F_t| — a unit
    vector along that residue, different in each summation order — so the second iterates part.  Both
    restatements converge (optimal; 61 and 39 iterations)."""
    prob, x0, mass = _testbasic("testCoMPlanner")
    c1 = pyoracle.solve(prob.desc(), x0, mass, max_iter=1)
    h1 = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), max_iter=1,
                         evaluator=OracleBatchEvaluator(prob, 1), hessian="limited-memory")
    assert np.abs(c1["x"] - h1.x[0].numpy()).max() <= 1e-12
    x = c1["x"]
    N = (x.shape[0] - 3) // 9
    ft = []
    for i in range(N):
        F, nv = x[3 + 9 * i: 6 + 9 * i], x[9 + 9 * i: 12 + 9 * i]
        if abs(F.dot(nv)) > 1e-3:
            ft.append(np.linalg.norm(F - F.dot(nv) * nv))
    assert ft and max(ft) < 1e-20  # loaded contacts with tangential forces at the rounding level
    c = pyoracle.solve(prob.desc(), x0, mass, max_iter=3000)
    h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), max_iter=3000,
                        evaluator=OracleBatchEvaluator(prob, 1), hessian="limited-memory")
    assert c["status"] == 0 and int(h.status[0]) == 0
    assert c["objective"] == pytest.approx(float(h.objective[0]), rel=1e-6)


def test_ipopt_jacobian_regularisation_on_the_simple_problem():
    """testSimpleProblem's systems are rank deficient at every iteration (one contact: the torque row about
    the force's own axis vanishes at the solution).  The restatements add delta_c to R's near-zero pivots
    with their own signs, which IPOPT does not: it regularises the (2,2) block, [[W, A^T], [A, -delta_c I]]
    (PDPerturbationHandler, delta_c = 1e-8 mu^0.25).  The compiled restatement has that form opt-in
    (cplo_set_jac_reg): there the problem converges (optimal in at most 20 iterations, measured 12, at an
    objective no worse) where the default form crawls to "acceptable" in 388 — the measured size of the
    difference, not the product's default."""
    prob, x0, mass = _testbasic("testSimpleProblem")
    d = pyoracle.solve(prob.desc(), x0, mass, max_iter=3000)
    pyoracle.set_jac_reg(True)
    try:
        r = pyoracle.solve(prob.desc(), x0, mass, max_iter=3000)
    finally:
        pyoracle.set_jac_reg(False)
    assert d["status"] == 1 and d["iterations"] == 388
    assert r["status"] == 0 and r["iterations"] <= 20
    assert r["objective"] <= d["objective"] * (1.0 + 1e-12)
    # the host restatement's opt-in form (batch_ipm_solve(jacobian_regularization="ipopt")): the same
    # iterations, the same point to rounding
    h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), max_iter=3000,
                        evaluator=OracleBatchEvaluator(prob, 1), hessian="limited-memory",
                        jacobian_regularization="ipopt")
    assert int(h.status[0]) == r["status"] and int(h.iterations[0]) == r["iterations"]
    np.testing.assert_allclose(h.x[0].numpy(), r["x"], rtol=0, atol=1e-9)


def _resto_case(k=0):
    import json
    import os

    from resto_cases import make

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resto_acc_cases.json")
    c = json.load(open(path))["cases"][k]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        prob = make(c["params"]).GetCplProblem()
    return prob, np.array(c["x0"]), c


@pytest.mark.parametrize("k", [0, 1])
def test_restoration_called_at_an_almost_feasible_point(k):
    """IPOPT's BacktrackingLineSearch calls no restoration phase at an almost feasible point (theta <=
    1e-2 tol): it restores the backup acceptable point and stops there as acceptable
    (RestoreAcceptablePoint), or without one the solve ends as a restoration failure ("Restoration phase
    called, but point is almost feasible").  Cases found by scripts/resto_acc_search.py
    (tests/golden/resto_acc_cases.json), where both restatements (and the engine,
    test_gpu_solve_engine.py) reach the branch: 0 — a ground scenario at tol 1e-6, where IPOPT's
    acceptable_tol 1e-6 stores no iterate (a restoration failure) and 1.78e-5 stores one (restored); 1 —
    a Superquadric scenario under IPOPT's defaults (tol 1e-8, acceptable_tol 1e-6: restored; with no
    backup point possible, a restoration failure).  The same iteration ends either way, at a different
    point.  (The degenerate trajectories part the restatements by rounding: the compiled one reaches the
    branch at iteration 129 / 1 414, the host one at 176 / 903, the device at 183 / 680; what is asserted
    is the branch and its outcome, per restatement.)"""
    import centroidalplanner_amd.batch_ipm as bi

    prob, x0, c = _resto_case(k)
    mass = prob.desc().mass
    nb, at = c["no_backup_tol"], c["acceptable_tol"]
    out = {}
    try:
        for a in (nb, at):
            pyoracle.set_acceptable_tol(a)
            pyoracle.resto_fail_events()
            out[a] = (pyoracle.solve(prob.desc(), x0, mass, tol=c["tol"], hessian=c["hessian"]),
                      pyoracle.resto_fail_events())
    finally:
        pyoracle.set_acceptable_tol(1e-6)
    (fail, ev0), (back, ev1) = out[nb], out[at]
    assert pyoracle.STATUS_NAMES[fail["status"]] == "resto_failed" and ev0 == (1, 0)
    assert pyoracle.STATUS_NAMES[back["status"]] == "acceptable" and ev1 == (1, 1)
    assert back["iterations"] == fail["iterations"] and back["objective"] != fail["objective"]
    hs = {}
    for a in (nb, at):
        log = []
        bi._DEBUG_EVENT = lambda name, mask: log.append(name)
        try:
            h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), tol=c["tol"],
                                max_iter=3000, evaluator=OracleBatchEvaluator(prob, 1), hessian=c["hessian"],
                                acceptable_tol=a)
        finally:
            bi._DEBUG_EVENT = None
        hs[a] = (int(h.status[0]), int(h.iterations[0]), float(h.objective[0]), "restore_acceptable_point" in log)
    (hst0, hit0, hobj0, hr0), (hst1, hit1, hobj1, hr1) = hs[nb], hs[at]
    assert hst0 == 4 and not hr0
    assert hst1 == 1 and hr1 and hit1 == hit0 and hobj1 != hobj0


def _watchdog_run(prob, X0, mass, hessian, trigger):
    """(compiled [(status, iterations, events)], host result, host events [B, 3]) with IPOPT's watchdog at
    `trigger` shortened steps (IPOPT: 10) in both restatements."""
    import centroidalplanner_amd.batch_ipm as bi

    B = X0.shape[0]
    pyoracle.set_watchdog(True)
    pyoracle.set_watchdog_params(trigger, 3)
    try:
        C = []
        for b in range(B):
            pyoracle.watchdog_events()
            r = pyoracle.solve(prob.desc(), X0[b], mass[b], max_iter=3000, hessian=hessian)
            C.append((r["status"], r["iterations"], pyoracle.watchdog_events(), r["x"]))
    finally:
        pyoracle.set_watchdog(False)
        pyoracle.set_watchdog_params(10, 3)
    ev = {k: np.zeros(B, dtype=np.int64) for k in ("watchdog_start", "watchdog_success", "watchdog_restore")}

    def dbg(name, mask):
        if name in ev:
            ev[name] += mask.numpy().astype(np.int64)

    bi._DEBUG_EVENT = dbg
    try:
        h = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob, 4),
                            max_iter=3000, hessian=hessian, watchdog=True, watchdog_trigger=trigger)
    finally:
        bi._DEBUG_EVENT = None
    return C, h, np.stack([ev["watchdog_start"], ev["watchdog_success"], ev["watchdog_restore"]], 1)


def test_watchdog_host_restatement_matches_compiled():
    """IPOPT's watchdog (BacktrackingLineSearch: watchdog_shortened_iter_trigger, watchdog_trial_iter_max 3)
    in the host restatement (batch_ipm_solve(watchdog=True), opt-in) against the compiled one
    (cplo_set_watchdog): at IPOPT's trigger of 10 it never starts on the solve workload (DESIGN.md section
    5), so the trigger is lowered to 1 here to exercise it.  Exact Hessian, 64 instances: the same status,
    iteration count and watchdog events (starts, successes, restorations of the kept iterate) per instance.
    L-BFGS instance 46 (the sample's one restore path: 6 starts, 2 successes, 4 restorations of the kept
    iterate and backtracking along its step): the same 59 iterations, events and point in both."""
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, 64, seed=21)
    C, h, ev = _watchdog_run(prob, X0, mass, "exact", 1)
    assert ev[:, 0].sum() >= 1
    for b in range(64):
        assert (int(h.status[b]), int(h.iterations[b])) == C[b][:2], b
        assert tuple(int(v) for v in ev[b]) == C[b][2], b
    C, h, ev = _watchdog_run(prob, X0[46:47], mass[46:47], "limited-memory", 1)
    assert C[0][2] == (6, 2, 4) and tuple(int(v) for v in ev[0]) == (6, 2, 4)
    assert int(h.status[0]) == C[0][0] == 0 and int(h.iterations[0]) == C[0][1] == 59
    np.testing.assert_allclose(h.x[0].numpy(), C[0][3], rtol=0, atol=1e-8)
