"""An independent single-instance NLP solver for cross-checks (TEST INFRASTRUCTURE): SciPy's
SLSQP over the TNLP hooks (get_bounds_info, eval_f, eval_grad_f, eval_g, eval_jac_g; the Jacobian
scattered from the CSR values with the (iRow, jCol) structure).  The batched solve loop's solutions
are compared against it (the problems are nonconvex: both find local optima)."""
from __future__ import annotations

import numpy as np

from centroidalplanner_amd._abi import INF
from centroidalplanner_amd.solver import SolveResult


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


def slsqp_solve(problem, evaluator, x0=None, tol: float = 1e-14, max_iter: int = 3000) -> SolveResult:
    ev = evaluator
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
