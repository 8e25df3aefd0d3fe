"""The compiled solve restatement (oracle/cpl_solve_host.c — the CPU baseline of bench.py's solve
legs) against the host path of the batched solver (batch_ipm.py over the oracle's callbacks): the
same iteration, so the same status, iteration count and restoration count, and the same point and
objective to rounding (the dense factorisations differ in summation order).  IPOPT itself is not in
the image; both restate its method (parity of the method: test_oracle_pinning.py)."""
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
