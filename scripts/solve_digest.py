"""Bitwise digest of the native engine's solve results (x, iterations, status) for the solve5 workload:
library builds compare bit for bit (CPL_LIB=<build> python scripts/solve_digest.py [--batch B]).
One JSON line per Hessian mode."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402
from centroidalplanner_amd.workload import solve_inputs, solve_problem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8192)
args = ap.parse_args()
prob = solve_problem().GetCplProblem()
dev = torch.device("cuda:0")
X0, mass = solve_inputs(prob, args.batch, seed=0xC910 + 5)
for hessian in ("limited-memory", "exact"):
    r = batch_ipm_solve(prob, torch.tensor(X0, device=dev), torch.tensor(mass, device=dev), max_iter=3000,
                        hessian=hessian)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (r.x, r.iterations, r.status):
        h.update(t.detach().cpu().contiguous().numpy().tobytes())
    print(json.dumps({"hessian": hessian, "batch": args.batch, "digest": h.hexdigest()[:16],
                      "iterations_sum": int(r.iterations.sum()), "solved": int((r.status <= 1).sum())}), flush=True)
