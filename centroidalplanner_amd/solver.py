"""Solve() plumbing of the facade: a host NLP driver over the GPU callbacks.

The reference drives each solve with ifopt::IpoptSolver (src/CentroidalPlanner.cpp:22-34).  IPOPT
is not in this image.  Two drivers consume the same TNLP hooks (get_bounds_info, eval_f,
eval_grad_f, eval_g, eval_jac_g; the Jacobian scattered from the CSR values with the (iRow, jCol)
structure):
  * method="slsqp" (default): SciPy's SLSQP, one instance;
  * method="ipm": the batched interior-point solve loop (batch_ipm.py, IPOPT's method) on a batch
    of one — the driver of the 8,192-instance solves, here from the problem's current variables
    (x = 0 initially, as the reference's IPOPT start point).  It takes rank-deficient equality
    Jacobians (TestBasic's single-contact problem), which SLSQP cannot.
Evaluators expose ``eval_batch(X[B, n]) -> {f, grad, g, jac}`` (host arrays); None = the GPU kernel.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._abi import INF


class TorchEvaluator:
    """Batched callbacks on the GPU through CplProblem.eval_batch (host arrays in and out)."""

    def __init__(self, problem):
        import torch

        self.problem = problem
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())

    def eval_batch(self, X):
        t = self.torch.as_tensor(np.ascontiguousarray(np.atleast_2d(X), dtype=np.float64), device=self.dev)
        out = self.problem.eval_batch(t, outputs=("g", "jac", "f", "grad"))
        return {k: v.cpu().numpy() for k, v in out.items()}


class _HostBatchEvaluator:
    """An eval_batch(X) evaluator as batch_ipm's callback (CPU tensors in and out)."""

    def __init__(self, ev):
        self.ev = ev

    def __call__(self, X, mass, outputs=("g", "jac", "f", "grad")):
        import torch

        o = self.ev.eval_batch(X.cpu().numpy())
        return {k: torch.as_tensor(np.asarray(o[k]), device=X.device) for k in outputs}


def _ipm_solve(problem, evaluator, x0, tol, max_iter) -> SolveResult:
    """The batched solve loop on one instance: the GPU loop (HIP kernels, graph-captured) when no
    evaluator is given, else the same algorithm's host path over the evaluator's callbacks."""
    import torch

    from .batch_ipm import STATUS_ACCEPTABLE, batch_ipm_solve

    xl, xu, gl, gu = problem.get_bounds_info()
    x0 = np.clip(problem.get_starting_point() if x0 is None else np.asarray(x0, dtype=np.float64), xl, xu)
    if evaluator is None:
        X0 = torch.as_tensor(x0[None], device=torch.device("cuda", torch.cuda.current_device()))
        r = batch_ipm_solve(problem, X0, None, tol=max(tol, 1e-8), max_iter=max_iter)
    else:
        r = batch_ipm_solve(problem, torch.as_tensor(x0[None]), None, evaluator=_HostBatchEvaluator(evaluator),
                            tol=max(tol, 1e-8), max_iter=max_iter)
    x = r.x[0].cpu().numpy()
    st = int(r.status[0])
    problem.SetVariables(x)  # the next Solve warm-starts here, like the reference's persistent variables
    names = {0: "optimal", 1: "acceptable"}
    return SolveResult(x, st <= STATUS_ACCEPTABLE, names.get(st, f"status {st}"), int(r.iterations[0]),
                       float(r.primal_inf[0]))


@dataclass
class SolveResult:
    x: np.ndarray
    success: bool
    status: str
    iterations: int
    primal_inf: float


class _Cached:
    """One evaluation per distinct x (SLSQP asks for f, grad, g, jac at the same point)."""

    def __init__(self, ev, nan_jac_to_zero):
        self.ev, self.key, self.out, self.nan0 = ev, None, None, nan_jac_to_zero

    def __call__(self, x):
        k = x.tobytes()
        if k != self.key:
            o = self.ev.eval_batch(np.asarray(x, dtype=np.float64)[None, :])
            self.out = {q: v[0] for q, v in o.items()}
            if self.nan0:
                self.out["jac"] = np.nan_to_num(self.out["jac"], nan=0.0)
            self.key = k
        return self.out


def solve(problem, evaluator=None, x0: Optional[np.ndarray] = None, tol: float = 1e-14, max_iter: int = 3000,
          method: str = "slsqp") -> SolveResult:
    if method == "ipm":
        return _ipm_solve(problem, evaluator, x0, tol, max_iter)
    if method != "slsqp":
        raise ValueError("method must be 'slsqp' or 'ipm'")
    ev = evaluator if evaluator is not None else TorchEvaluator(problem)
    from scipy.optimize import minimize

    n, m, nnz = problem.get_nlp_info()
    iRow, jCol = problem.get_structure()
    xl, xu, gl, gu = problem.get_bounds_info()
    x0 = problem.get_starting_point() if x0 is None else np.asarray(x0, dtype=np.float64)
    x0 = np.clip(x0, xl, xu)
    at = _Cached(ev, nan_jac_to_zero=True)  # a cone at zero tangential force has a 0/0 Jacobian

    def J(x):
        A = np.zeros((m, n))
        A[iRow, jCol] = at(x)["jac"]
        return A

    eq = np.where(gl == gu)[0]
    up = np.where((gl != gu) & (gu < INF / 10))[0]
    lo = np.where((gl != gu) & (gl > -INF / 10))[0]
    cons = []
    if eq.size:
        cons.append({"type": "eq", "fun": lambda x: at(x)["g"][eq] - gu[eq], "jac": lambda x: J(x)[eq]})
    if up.size:
        cons.append({"type": "ineq", "fun": lambda x: gu[up] - at(x)["g"][up], "jac": lambda x: -J(x)[up]})
    if lo.size:
        cons.append({"type": "ineq", "fun": lambda x: at(x)["g"][lo] - gl[lo], "jac": lambda x: J(x)[lo]})
    res = minimize(lambda x: float(at(x)["f"]), x0, jac=lambda x: at(x)["grad"], bounds=list(zip(xl, xu)),
                   constraints=cons, method="SLSQP", options={"ftol": tol, "maxiter": max_iter})
    x = np.clip(res.x, xl, xu)
    g = at(x)["g"]
    viol = np.maximum(np.maximum(gl - g, g - gu), 0.0)
    problem.SetVariables(x)  # the next Solve warm-starts here, like the reference's persistent variables
    return SolveResult(x, bool(res.success), str(res.message), int(res.nit), float(viol.max(initial=0.0)))
