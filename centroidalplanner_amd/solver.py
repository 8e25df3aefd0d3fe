"""Solve() plumbing of the facade: the batched interior-point solve loop on a batch of one.

The reference drives each solve with ifopt::IpoptSolver (src/CentroidalPlanner.cpp:22-34): IPOPT
with IFOPT's defaults — exact constraint Jacobian, limited-memory Hessian, max_iter 3000, tol 1e-8
— from the problem's current variables (x = 0 initially, src/Variable3D.cpp:8-10).  IPOPT is not in
this image; the same method runs here as the batched solve loop (batch_ipm.py, the driver of the
8,192-instance solves) with B = 1: on the GPU (HIP kernels, the iteration captured as a HIP graph)
when no evaluator is given, else on the host over the evaluator's callbacks (tests inject the
oracle).  Like IFOPT's solver, a run that ends without convergence does not throw: the last iterate
is kept (src/CentroidalPlanner.cpp:29-33) and `success` says how it ended (the engine's opt-in
best-feasible fallback is off here, as IPOPT returns its last iterate).  IPOPT's gradient-based NLP
scaling is on, as in the reference.  Where the start point's constraint Jacobian has NaN entries
(FrictionCone's 0/0 at a zero tangential force, e.g. x = 0) the loop takes them as 0; the solve's own
start-point evaluation counts them (cpl_solver_nan_jacobian — no extra evaluation), the count is
returned (`nan_jacobian_at_start`) and a RuntimeWarning says so — IPOPT would receive the NaNs.
Evaluators expose ``eval_batch(X[B, n]) -> {f, grad, g, jac}`` (host arrays).
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class SolveResult:
    x: np.ndarray
    success: bool
    status: str
    iterations: int
    primal_inf: float
    derivative_report: Optional[dict] = None  # derivative_test = "first-order" (cpl_derivative_test)
    fallback: bool = False  # not converged, last iterate infeasible: x is the best feasible iterate instead
    # Jacobian entries NaN at the start point (FrictionCone's 0/0 where F_t = 0,
    # src/Constraints/FrictionCone.cpp:85-87, e.g. x = 0): IPOPT would receive NaN, the loop takes 0
    nan_jacobian_at_start: int = 0


class _HostBatchEvaluator:
    """An eval_batch(X) evaluator as batch_ipm's callback (CPU tensors in and out); forwards an
    analytic `hessian(X, y, free)` when the evaluator has one."""

    def __init__(self, ev):
        self.ev = ev
        if hasattr(ev, "hessian"):
            self.hessian = self._hessian

    def __call__(self, X, mass, outputs=("g", "jac", "f", "grad")):
        import torch

        o = self.ev.eval_batch(X.cpu().numpy())
        return {k: torch.as_tensor(np.asarray(o[k]), device=X.device) for k in outputs}

    def _hessian(self, X, y, free, zero_cost=False):
        import torch

        H = self.ev.hessian(X.cpu().numpy(), y.cpu().numpy(), free.cpu().numpy(), zero_cost=zero_cost)
        return None if H is None else torch.as_tensor(np.asarray(H), device=X.device)


def solve(problem, evaluator=None, x0: Optional[np.ndarray] = None, tol: float = 1e-8, max_iter: int = 3000,
          hessian: str = "limited-memory", derivative_test: str = "none",
          jacobian_regularization: str = "pivot") -> SolveResult:
    """One instance through the batched solve loop.  hessian: "limited-memory" (IFOPT's default, as
    the reference runs) or "exact" (the analytic Lagrangian Hessian).  derivative_test:
    "first-order" runs IPOPT's first-order derivative checker at the start point first, as the
    reference's solver option does (src/CentroidalPlanner.cpp:26); its report is returned.
    jacobian_regularization: "pivot" (default) or "ipopt" (batch_ipm_solve's option)."""
    if derivative_test not in ("none", "first-order"):
        raise ValueError(f"derivative_test must be 'none' or 'first-order', not {derivative_test!r}")
    import torch

    from .batch_ipm import STATUS_ACCEPTABLE, STATUS_NAMES, batch_ipm_solve

    xl, xu, _, _ = problem.get_bounds_info()
    x0 = np.clip(problem.get_starting_point() if x0 is None else np.asarray(x0, dtype=np.float64), xl, xu)
    report = None
    if evaluator is None:
        X0 = torch.as_tensor(x0[None], device=torch.device("cuda", torch.cuda.current_device()))
        if derivative_test == "first-order":
            report = problem.derivative_test(X0)
        r = batch_ipm_solve(problem, X0, None, tol=tol, max_iter=max_iter, hessian=hessian,
                            jacobian_regularization=jacobian_regularization)
    else:
        r = batch_ipm_solve(problem, torch.as_tensor(x0[None]), None, evaluator=_HostBatchEvaluator(evaluator),
                            tol=tol, max_iter=max_iter, hessian=hessian,
                            jacobian_regularization=jacobian_regularization)
    # the NaN Jacobian entries the solve's own start-point evaluation met (cpl_solver_nan_jacobian)
    nan0 = int(r.nan_jacobian[0])
    if nan0:
        warnings.warn(f"{nan0} constraint Jacobian entries are NaN at the start point (FrictionCone's 0/0 where "
                      f"a contact's tangential force is 0, src/Constraints/FrictionCone.cpp:85-87); IPOPT would "
                      f"receive them as NaN, this solve takes them as 0 (a subgradient)", RuntimeWarning, stacklevel=2)
    x = r.x[0].cpu().numpy()
    st = int(r.status[0])
    problem.SetVariables(x)  # the next Solve warm-starts here, like the reference's persistent variables
    return SolveResult(x, st <= STATUS_ACCEPTABLE, STATUS_NAMES.get(st, f"status {st}"), int(r.iterations[0]),
                       float(r.primal_inf[0]), report, bool(r.fallback[0]) if r.fallback is not None else False,
                       nan0)
