"""Trace the batched solve on the GPU (kernel callbacks) for a few instances (debug aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from centroidalplanner_amd.batch_ipm import batch_ipm_solve
from centroidalplanner_amd.workload import solve_inputs, solve_problem
prob = solve_problem().GetCplProblem()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
X0, mass = solve_inputs(prob, B, seed=11)
dev = torch.device(sys.argv[2] if len(sys.argv) > 2 else "cuda:0")
r = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), max_iter=12, verbose=2)
print(r.status.tolist(), r.iterations.tolist(), r.objective.tolist())
