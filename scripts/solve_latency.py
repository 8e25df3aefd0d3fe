"""Single-instance solve latency of the native engine (what CentroidalPlanner::Solve() costs per call):
B = 1 solves of the solve5 workload's first instances, both Hessian modes, plus a B = 64 batch for
the per-instance amortisation.

python scripts/solve_latency.py [--reps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402
from centroidalplanner_amd.workload import solve_inputs, solve_problem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--only", default="", help="run one case, e.g. limited-memory:1 (for a kernel trace)")
ap.add_argument("--ls-kernel", type=int, default=2, help="the engine's ls_kernel option (0 / 1 / 2)")
ap.add_argument("--variant", type=int, default=0, help="eval kernel variant (cpl_set_tuning), 0 = auto")
ap.add_argument("--no-graph", action="store_true", help="launch the iteration's kernels directly (no HIP graph)")
args = ap.parse_args()
if args.variant:
    from centroidalplanner_amd import _abi  # noqa: E402

    _abi.check(_abi.lib.cpl_set_tuning(args.variant, 0, 256, 1, 0))

prob = solve_problem().GetCplProblem()
dev = torch.device("cuda:0")
X0, mass = solve_inputs(prob, 64, seed=0xC910 + 5)
out = {}
cases = [(h, B) for h in ("limited-memory", "exact") for B in (1, 64)]
if args.only:
    h, b = args.only.split(":")
    cases = [(h, int(b))]
for hessian, B in cases:
    if True:
        Xt, mt = torch.tensor(X0[:B], device=dev), torch.tensor(mass[:B], device=dev)
        r = batch_ipm_solve(prob, Xt, mt, max_iter=1000, hessian=hessian, ls_kernel=args.ls_kernel,
                            graph=not args.no_graph)  # warm: engine + graphs
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            r = batch_ipm_solve(prob, Xt, mt, max_iter=1000, hessian=hessian, ls_kernel=args.ls_kernel,
                            graph=not args.no_graph)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        its = r.iterations.double()
        out[f"{hessian}_B{B}"] = {"ms_per_solve_call": dt * 1e3, "ms_per_instance": dt * 1e3 / B,
                                  "lockstep_iterations": r.iterations_run, "iterations_mean": float(its.mean()),
                                  "us_per_lockstep_iteration": dt * 1e6 / max(1, r.iterations_run),
                                  "solved": int((r.status <= 1).sum())}
print(json.dumps(out), flush=True)
