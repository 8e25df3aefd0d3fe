"""The device engine on the RestoreAcceptablePoint candidates of scripts/resto_acc_search.py
(scripts/resto_acc_candidates.json: TestBasic-like scenarios whose compiled-restatement solve
calls the restoration phase at an almost feasible point).  Per candidate: the engine with no backup
point possible (acceptable_tol 1e-300) — its status and iteration count — and, where that ended in
the almost-feasible restoration failure, a sweep of acceptable_tol: a value at which the same
iteration ends "acceptable" at a different (the restored) point is the branch firing on the device.
GPU.

python scripts/resto_acc_gpu_probe.py [candidates.json] > out.jsonl
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]

from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402
from resto_acc_search import case  # noqa: E402


def solve(prob, x0, tol, at, hessian):
    dev = torch.device("cuda:0")
    r = batch_ipm_solve(prob, torch.as_tensor(x0[None], device=dev),
                        torch.as_tensor(np.array([prob.desc().mass]), device=dev), tol=tol, max_iter=3000,
                        acceptable_tol=at, hessian=hessian)
    return int(r.status[0]), int(r.iterations[0]), float(r.objective[0])


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scripts", "resto_acc_candidates.json")
    cands = json.load(open(path))
    t0 = time.time()
    for c in cands:
        P, cpl, x0 = case(c["seed"])
        assert P == c["params"], "resto_acc_search.draw changed"
        prob = cpl.GetCplProblem()
        st, it, obj = solve(prob, x0, c["tol"], 1e-300, c["hessian"])
        out = {"seed": c["seed"], "tol": c["tol"], "hessian": c["hessian"], "no_backup": [st, it, obj], "restored_at": []}
        if st == 4:
            for at in np.logspace(-10, 2, 25):
                s2, i2, o2 = solve(prob, x0, c["tol"], float(at), c["hessian"])
                if s2 == 1 and i2 == it and o2 != obj:
                    out["restored_at"].append([float(at), i2, o2])
        out["seconds"] = round(time.time() - t0, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
