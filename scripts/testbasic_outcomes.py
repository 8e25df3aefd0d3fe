"""TestBasic's four scenarios (tests/TestBasic.cpp of the reference) solved by CentroidalPlanner::Solve()
from the reference's start point x = 0 under IFOPT's defaults (limited-memory Hessian, max_iter 3000):
per scenario and backend (the GPU engine; "oracle": the host restatement over the CPU oracle's
callbacks) the outcome, the iteration count, whether the best-feasible fallback was taken, the NaN
Jacobian entries at the start, the returned point's TestBasic quantities (force / torque balance
errors, worst cone value) and the wall time.  One JSON line per run.

usage: python scripts/testbasic_outcomes.py [gpu|oracle|both] [pivot|ipopt] > out.jsonl
(the second argument: the facade's solver_jacobian_regularization; default: the facade's own, pivot)
"""
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from centroidalplanner_amd import CentroidalPlanner, CoMPlanner, Ground, Superquadric  # noqa: E402

NAMES = ["contact1", "contact2", "contact3", "contact4"]
MASS, G = 100.0, -9.81
WRENCH = np.array([100.0, 0.0, 0.0, 0.0, 0.0, 100.0])


def simple():  # TestBasic.cpp:28-61
    env = Ground()
    env.SetGroundZ(0.1)
    return CentroidalPlanner(["contact1"], MASS, env), np.zeros(6), 1.0


def ground():  # TestBasic.cpp:64-135
    env = Ground()
    env.SetGroundZ(0.1)
    env.SetMu(0.5)
    cpl = CentroidalPlanner(NAMES, MASS, env)
    cpl.SetCoMWeight(2.0)
    cpl.SetForceWeight(0.0)
    for c in NAMES:
        cpl.SetPosBounds(c, np.array([-0.3, -0.3, 0.0]), np.array([0.3, 0.3, 1.0]))
    cpl.SetManipulationWrench(WRENCH)
    return cpl, WRENCH, 0.5


def superquadric():  # TestBasic.cpp:138-222
    env = Superquadric()
    env.SetMu(0.5)
    env.SetParameters(np.array([0.0, 0.0, 1.0]), np.array([0.3, 0.3, 10.0]), np.array([10.0, 10.0, 10.0]))
    cpl = CentroidalPlanner(NAMES, MASS, env)
    cpl.SetForceWeight(0.0)
    for c in NAMES:
        cpl.SetPosBounds(c, np.array([-0.5, -0.5, 0.5]), np.array([0.5, 0.5, 1.5]))
    cpl.SetManipulationWrench(WRENCH)
    return cpl, WRENCH, 0.5


def com_planner():  # TestBasic.cpp:225-292
    cpl = CoMPlanner(NAMES, MASS)
    cpl.SetMu(0.5)
    for c, p in zip(NAMES, ([1.0, 1.0, 0.0], [-1.0, 1.0, 0.0], [-1.0, -1.0, 0.0], [1.0, -1.0, 0.0])):
        cpl.SetContactPosition(c, p)
    cpl.SetLiftingContact("contact4")
    for c in NAMES:
        cpl.SetForceThreshold(c, 20.0)
    return cpl, np.zeros(6), 0.5


class _Oracle:
    def __init__(self, prob):
        import pyoracle

        self.prob, self.po = prob, pyoracle

    def eval_batch(self, X):
        return self.po.eval_batch(self.prob.desc(), np.atleast_2d(X), outputs=("g", "jac", "f", "grad"), nthreads=1)


def run(name, make, backend, jac_reg=None):
    cpl, wrench, mu = make()
    inner = getattr(cpl, "_cp", cpl)  # (CoMPlanner wraps a CentroidalPlanner)
    if jac_reg is not None:
        inner.solver_jacobian_regularization = jac_reg
    jac_reg = inner.solver_jacobian_regularization
    if backend == "oracle":
        cpl.evaluator = _Oracle(cpl.GetCplProblem())
    t0 = time.perf_counter()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        sol = cpl.Solve()
    dt = time.perf_counter() - t0
    F_sum, T_sum, cone = np.zeros(3), np.zeros(3), -np.inf
    for v in sol.contact_values_map.values():
        F, n = v.force_value, v.normal_value
        F_sum += F
        T_sum += np.cross(v.position_value - sol.com_sol, F)
        cone = max(cone, float(-F.dot(n)), float(np.linalg.norm(F - n.dot(F) * n) - mu * F.dot(n)))
    fb = F_sum - np.array([wrench[0], wrench[1], -MASS * G + wrench[2]])
    return {"scenario": name, "backend": backend, "jacobian_regularization": jac_reg, "status": sol.message, "iterations": sol.iterations,
            "fallback": bool(sol.fallback), "nan_jacobian_at_start": int(sol.nan_jacobian_at_start),
            "force_balance_err": float(np.abs(fb).max()), "torque_balance_err": float(np.abs(T_sum - wrench[3:]).max()),
            "worst_cone_value": cone, "seconds": dt}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "gpu"
    backends = ["gpu", "oracle"] if which == "both" else [which]
    jac_reg = sys.argv[2] if len(sys.argv) > 2 else None
    for backend in backends:
        for name, make in (("testSimpleProblem", simple), ("testGroundEnv", ground),
                           ("testSuperquadricEnv", superquadric), ("testCoMPlanner", com_planner)):
            print(json.dumps(run(name, make, backend, jac_reg)), flush=True)


if __name__ == "__main__":
    main()
