"""What IPOPT's Jacobian regularisation costs the engine (cpl_solve_options.jacobian_regularization = 1:
an augmented-system launch after every KKT call, the second-order corrections stepwise): wall time per
solve call, pivot vs ipopt, at B = 1 (the facade's Solve()) and B = 8 192 (the solve workload), and
whether the results are bitwise the pivot form's (they are whenever no system loses rank)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402
from centroidalplanner_amd.workload import solve_inputs, solve_problem  # noqa: E402

prob = solve_problem().GetCplProblem()
dev = torch.device("cuda:0")
for B, reps in ((1, 7), (64, 5), (8192, 3)):
    X0, mass = solve_inputs(prob, B)
    X0t, mt = torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev)
    for hess in ("limited-memory", "exact"):
        res = {}
        for jr in ("pivot", "ipopt", "pivot", "ipopt"):  # interleaved, the first of each a warm-up
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = batch_ipm_solve(prob, X0t, mt, max_iter=3000, hessian=hess, jacobian_regularization=jr)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            res[jr] = (statistics.median(ts), r)
        same = bool(torch.equal(res["pivot"][1].x, res["ipopt"][1].x)
                    and torch.equal(res["pivot"][1].iterations, res["ipopt"][1].iterations))
        print(json.dumps({"batch": B, "hessian": hess, "ms_pivot": res["pivot"][0] * 1e3,
                          "ms_ipopt": res["ipopt"][0] * 1e3, "ratio": res["ipopt"][0] / res["pivot"][0],
                          "bitwise_equal": same}), flush=True)
