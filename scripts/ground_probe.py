"""Debug aid: TestBasic's ground scenario (tests/TestBasic.cpp:64-135 of the reference) solved from x = 0
on the device engine, stopped at a grid of max_iter values — the run is deterministic, so each stop
is a point of the same trajectory.  Prints, per stop, the status, the returned point's primal
infeasibility, objective and TestBasic's checks (force / torque balance, worst cone value).

usage: python scripts/ground_probe.py [hessian] [grid spec "a:b:s,..."] > out.jsonl
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from centroidalplanner_amd import CentroidalPlanner, Ground  # noqa: E402
from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402


def ground_planner():
    names = ["contact1", "contact2", "contact3", "contact4"]
    env = Ground()
    env.SetGroundZ(0.1)
    env.SetMu(0.5)
    cpl = CentroidalPlanner(names, 100.0, env)
    cpl.SetCoMWeight(2.0)
    cpl.SetForceWeight(0.0)
    for c in names:
        cpl.SetPosBounds(c, np.array([-0.3, -0.3, 0.0]), np.array([0.3, 0.3, 1.0]))
    w = np.zeros(6)
    w[0] = 100.0
    w[5] = 100.0
    cpl.SetManipulationWrench(w)
    return cpl, w


def checks(x, w, mu=0.5, N=4):
    c = x[:3]
    Fs, Ts, cone, push = np.zeros(3), np.zeros(3), [], []
    for i in range(N):
        F, p, n = x[3 + 9 * i:6 + 9 * i], x[6 + 9 * i:9 + 9 * i], x[9 + 9 * i:12 + 9 * i]
        Fs += F
        Ts += np.cross(p - c, F)
        cone.append(float(np.linalg.norm(F - n.dot(F) * n) - mu * F.dot(n)))
        push.append(float(-F.dot(n)))
    fb = Fs - np.array([w[0], w[1], 981.0 + w[2]])
    tb = Ts - w[3:]
    return {"fbal": float(np.abs(fb).max()), "tbal": float(np.abs(tb).max()), "cone": cone, "push": push,
            "Fn": [float(x[5 + 9 * i]) for i in range(N)]}


def main():
    hess = sys.argv[1] if len(sys.argv) > 1 else "limited-memory"
    spec = sys.argv[2] if len(sys.argv) > 2 else "100:3001:100"
    grid = []
    for part in spec.split(","):
        a, b, s = (int(v) for v in part.split(":"))
        grid += list(range(a, b, s))
    cpl, w = ground_planner()
    prob = cpl.GetCplProblem()
    dev = torch.device("cuda:0")
    X0 = torch.zeros(1, prob.get_nlp_info()[0], dtype=torch.float64, device=dev)
    xl, xu, _, _ = prob.get_bounds_info()
    X0 = torch.as_tensor(np.clip(X0.cpu().numpy(), xl, xu), device=dev)
    for k in grid:
        r = batch_ipm_solve(prob, X0, None, max_iter=k, hessian=hess)
        x = r.x[0].cpu().numpy()
        rec = {"max_iter": k, "status": int(r.status[0]), "iters": int(r.iterations[0]),
               "pinf": float(r.primal_inf[0]), "dinf": float(r.dual_inf[0]), "obj": float(r.objective[0]),
               "resto": int(r.restorations[0]) if r.restorations is not None else None,
               "fallback": bool(r.fallback[0]) if r.fallback is not None else None}
        rec.update(checks(x, w))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
