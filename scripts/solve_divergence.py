"""Where the compiled solve restatement (oracle/cpl_solve_host.c, the solve legs' CPU baseline) and the
host restatement (batch_ipm.py over the oracle's callbacks) part on one instance: both run with
max_iter = k for k = 1, 2, ... and the returned points (the k-th iterate, projected onto the bounds)
compared.  Prints, per k, the largest |x_c - x_h| and the two statuses; stops at the first k whose
difference exceeds --tol (or at --kmax).  CPU only.
    python scripts/solve_divergence.py [testCoMPlanner|testSuperquadricEnv|testGroundEnv|testSimpleProblem|solve5:<b>]
"""
import argparse
import json
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

import pyoracle  # noqa: E402
from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402
from test_batch_solve import OracleBatchEvaluator  # noqa: E402
import testbasic_outcomes as tb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("scenario", nargs="?", default="testCoMPlanner")
ap.add_argument("--kmax", type=int, default=200)
ap.add_argument("--tol", type=float, default=1e-9)
ap.add_argument("--hessian", default="limited-memory")
ap.add_argument("--start", type=int, default=1)
args = ap.parse_args()

if args.scenario.startswith("solve5"):
    from centroidalplanner_amd.workload import solve_inputs, solve_problem

    b = int(args.scenario.split(":")[1]) if ":" in args.scenario else 0
    prob = solve_problem().GetCplProblem()
    X0, M = solve_inputs(prob, b + 1)
    x0, mass = X0[b], float(M[b])
else:
    make = {"testSimpleProblem": tb.simple, "testGroundEnv": tb.ground, "testSuperquadricEnv": tb.superquadric,
            "testCoMPlanner": tb.com_planner}[args.scenario]
    cpl, _, _ = make()
    prob = cpl.GetCplProblem()
    xl, xu, _, _ = prob.get_bounds_info()
    x0 = np.clip(prob.get_starting_point(), xl, xu)
    mass = float(prob.desc().mass)

ev = OracleBatchEvaluator(prob, 1)
for k in range(args.start, args.kmax + 1):
    c = pyoracle.solve(prob.desc(), x0, mass, max_iter=k, hessian=args.hessian)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])), max_iter=k,
                            evaluator=ev, hessian=args.hessian)
    d = float(np.abs(c["x"] - h.x[0].numpy()).max())
    rec = {"k": k, "max_abs_dx": d, "status_c": c["status"], "status_h": int(h.status[0]), "it_c": c["iterations"],
           "it_h": int(h.iterations[0]), "resto_c": c["restorations"], "resto_h": int(h.restorations[0]),
           "f_c": c["objective"], "f_h": float(h.objective[0])}
    print(json.dumps(rec), flush=True)
    if d > args.tol or c["status"] != int(h.status[0]) or (c["status"] <= 1 and int(h.status[0]) <= 1):
        break
