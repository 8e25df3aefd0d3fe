"""Diagnostics: the regularised form on TestBasic's ground scenario, device against host per iterate."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_batch_solve import OracleBatchEvaluator  # noqa: E402
from test_oracle_solve import _testbasic  # noqa: E402

from centroidalplanner_amd.batch_ipm import batch_ipm_solve  # noqa: E402

prob, x0, _ = _testbasic("testGroundEnv")
B = 4
mass = np.array([100.0, 90.0, 110.0, 125.0])
X0 = np.tile(x0, (B, 1))
dev = torch.device("cuda:0")
for hess in ("exact", "limited-memory"):
    for extra in ({}, {"max_soc": 0}, {"ls_kernel": 0}):
        hs = {}
        for k in (1, 2, 3):
            kw = dict(max_iter=k, hessian=hess, jacobian_regularization="ipopt", **extra)
            g = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), **kw)
            h = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob, B),
                                **kw)
            hs[k] = h.x
            gx = g.x.cpu()
            row = [f"{float((gx[b] - h.x[b]).abs().max()):.2e}" for b in range(B)]
            prev = [f"{float((gx[b] - hs[k - 1][b]).abs().max()):.2e}" for b in range(B)] if k > 1 else "-"
            print(hess, extra, "k", k, "dev-host", row, "dev-host(k-1)", prev, "status", g.status.tolist(), h.status.tolist(),
                  flush=True)
