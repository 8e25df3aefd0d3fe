"""Primal-dual interior-point NLP solver (IPOPT's algorithm, dense, one instance) over the TNLP hooks.

The reference solves with IPOPT through ifopt::IpoptSolver (src/CentroidalPlanner.cpp:22-34);
IPOPT is not available in this image, so this module restates the parts of IPOPT's method this
problem class needs (Wächter & Biegler 2006):
  * barrier formulation over the free variables and one slack per inequality row
    (g_I(x) - s = 0, s in [g_l, g_u]); fixed variables (x_l == x_u, e.g. CoMPlanner's contact
    positions and normals) are removed, as IPOPT's fixed_variable_treatment=make_parameter;
  * Newton steps on the primal-dual KKT system with inertia correction: delta_w on the Hessian
    block until the inertia is (n+, m-, 0), delta_c on the constraint block when the Jacobian is
    rank-deficient (the single-contact problem is: a torque about the force line is never
    produced), the inertia read off scipy's LDL^T factorisation;
  * fraction-to-the-boundary rule, monotone barrier update, backtracking line search on the
    l1 exact-penalty merit function.
The Hessian of the Lagrangian is a central finite difference of its exact gradient
grad f + J^T y; the 2n perturbed points are evaluated as ONE batch (``evaluator.eval_batch``), which
is how the GPU path wants to be called.

The evaluator is any object with ``eval_batch(X[B, n]) -> {"f","grad","g","jac"}`` host arrays.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
from scipy.linalg import ldl

from ._abi import INF

BIG = INF / 10.0  # |bound| >= 1e19 is infinite (IPOPT nlp_lower/upper_bound_inf)


@dataclass
class IpmResult:
    x: np.ndarray
    y: np.ndarray
    success: bool
    status: str
    iterations: int
    primal_inf: float
    dual_inf: float
    objective: float


class TorchEvaluator:
    """Batched callbacks on the GPU through CplProblem.eval_batch (copies in / out per batch)."""

    def __init__(self, problem):
        import torch

        self.problem = problem
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())

    def eval_batch(self, X):
        t = self.torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=self.dev)
        out = self.problem.eval_batch(t, outputs=("g", "jac", "f", "grad"))
        return {k: v.cpu().numpy() for k, v in out.items()}


def _inertia(D, tol=0.0):
    """(n_pos, n_neg, n_zero) of the block-diagonal D of an LDL^T factorisation."""
    pos = neg = zero = 0
    i, k = 0, D.shape[0]
    while i < k:
        if i + 1 < k and D[i + 1, i] != 0.0:
            ev = np.linalg.eigvalsh(D[i:i + 2, i:i + 2])
            for e in ev:
                if e > tol:
                    pos += 1
                elif e < -tol:
                    neg += 1
                else:
                    zero += 1
            i += 2
        else:
            e = D[i, i]
            if e > tol:
                pos += 1
            elif e < -tol:
                neg += 1
            else:
                zero += 1
            i += 1
    return pos, neg, zero


def ipm_solve(problem, evaluator, x0: Optional[np.ndarray] = None, tol: float = 1e-9, max_iter: int = 300,
              mu0: float = 0.1, fd_step: float = 1e-6, nan_jac_to_zero: bool = True, verbose: bool = False
              ) -> IpmResult:
    n, m, nnz = problem.get_nlp_info()
    iRow, jCol = problem.get_structure()
    xl, xu, gl, gu = problem.get_bounds_info()
    x = problem.get_starting_point() if x0 is None else np.asarray(x0, dtype=np.float64).copy()

    fixed = np.abs(xu - xl) <= 1e-14 * np.maximum(1.0, np.abs(xl))
    free = np.where(~fixed)[0]
    x[fixed] = xl[fixed]
    nf = free.size
    E = np.where(gl == gu)[0]
    I = np.where(gl != gu)[0]
    nI = I.size
    nw = nf + nI                      # unknowns w = [x_free, s]

    def evals(X):
        out = evaluator.eval_batch(np.atleast_2d(X))
        if nan_jac_to_zero:
            out["jac"] = np.nan_to_num(out["jac"], nan=0.0)
        return out

    def dense_J(jv):
        J = np.zeros((m, n))
        J[iRow, jCol] = jv
        return J

    # bounds of w, bound push (IPOPT bound_push = bound_frac = 1e-2)
    wl = np.concatenate([xl[free], np.where(gl[I] > -BIG, gl[I], -np.inf)])
    wu = np.concatenate([xu[free], np.where(gu[I] < BIG, gu[I], np.inf)])
    hasL, hasU = np.isfinite(wl), np.isfinite(wu)

    def push(v):
        v = v.copy()
        k1 = 1e-2
        pl = np.where(hasL, np.minimum(k1 * np.maximum(1.0, np.abs(wl)), k1 * np.where(hasU, wu - wl, np.inf)), 0.0)
        pu = np.where(hasU, np.minimum(k1 * np.maximum(1.0, np.abs(wu)), k1 * np.where(hasL, wu - wl, np.inf)), 0.0)
        v = np.where(hasL, np.maximum(v, wl + pl), v)
        v = np.where(hasU, np.minimum(v, wu - pu), v)
        return v

    ev0 = evals(x)
    w = np.concatenate([x[free], ev0["g"][0][I]])
    w = push(w)

    def unpack(wv):
        xx = x.copy()
        xx[free] = wv[:nf]
        return xx, wv[nf:]

    def cons(g, s):
        c = np.empty(m)
        c[E] = g[E] - gl[E]
        c[I] = g[I] - s
        return c

    def jac_w(J):
        A = np.zeros((m, nw))
        A[:, :nf] = J[:, free]
        A[I, nf + np.arange(nI)] = -1.0
        return A

    mu = mu0
    zL = np.where(hasL, mu / np.maximum(w - wl, 1e-300), 0.0)
    zU = np.where(hasU, mu / np.maximum(wu - w, 1e-300), 0.0)
    y = np.zeros(m)
    delta_w_last = 0.0
    tau_min = 0.99
    it = 0
    status = "max_iter"
    f = g = J = grad = None
    nu = 1.0

    def barrier_obj(fv, wv, muv):
        with np.errstate(divide="ignore", invalid="ignore"):
            bl = np.where(hasL, np.log(np.where(hasL, wv - wl, 1.0)), 0.0)
            bu = np.where(hasU, np.log(np.where(hasU, wu - wv, 1.0)), 0.0)
        return fv - muv * (bl.sum() + bu.sum())

    for it in range(max_iter + 1):
        xx, s = unpack(w)
        # ---- evaluate at x and at the 2*nf finite-difference points of the Lagrangian gradient
        hstep = fd_step * np.maximum(1.0, np.abs(xx[free]))
        P = np.repeat(xx[None, :], 1 + 2 * nf, axis=0)
        P[1 + np.arange(nf), free] += hstep
        P[1 + nf + np.arange(nf), free] -= hstep
        out = evals(P)
        f, grad, g, J = out["f"][0], out["grad"][0], out["g"][0], dense_J(out["jac"][0])
        c = cons(g, s)
        A = jac_w(J)
        gradw = np.concatenate([grad[free], np.zeros(nI)])
        # least-squares multiplier estimate at the start (IPOPT: constr_mult_init)
        if it == 0:
            ls = np.linalg.lstsq(A.T, -(gradw - zL + zU), rcond=None)[0]
            y = ls if np.abs(ls).max() <= 1e3 else np.zeros(m)
        dual = gradw + A.T @ y - zL + zU
        compL = np.where(hasL, (w - wl) * zL, 0.0)
        compU = np.where(hasU, (wu - w) * zU, 0.0)
        s_max = 100.0
        sd = max(s_max, (np.abs(y).sum() + np.abs(zL).sum() + np.abs(zU).sum()) / max(m + 2 * nw, 1)) / s_max
        sc = max(s_max, (np.abs(zL).sum() + np.abs(zU).sum()) / max(2 * nw, 1)) / s_max
        err0 = max(np.abs(dual).max() / sd, np.abs(c).max(), max(compL.max(initial=0), compU.max(initial=0)) / sc)
        if verbose:
            print(f"it {it:3d} f={f:.10g} inf_pr={np.abs(c).max():.2e} inf_du={np.abs(dual).max():.2e} mu={mu:.1e}")
        if err0 <= tol:
            status = "optimal"
            break
        if it == max_iter:
            break
        # barrier update (monotone Fiacco-McCormick)
        while True:
            errmu = max(np.abs(dual).max() / sd, np.abs(c).max(),
                        max(np.abs(compL - np.where(hasL, mu, 0)).max(initial=0),
                            np.abs(compU - np.where(hasU, mu, 0)).max(initial=0)) / sc)
            if errmu > 10.0 * mu or mu <= tol / 10.0:
                break
            mu = max(tol / 10.0, min(0.2 * mu, mu ** 1.5))
            tau_min = max(0.99, 1.0 - mu)
        # ---- Hessian of the Lagrangian over the free x (FD of grad f + J^T y)
        gp = out["grad"][1:1 + nf][:, free] + np.einsum("bmn,m->bn", np.stack([dense_J(v) for v in out["jac"][1:1 + nf]]), y)[:, free]
        gm = out["grad"][1 + nf:][:, free] + np.einsum("bmn,m->bn", np.stack([dense_J(v) for v in out["jac"][1 + nf:]]), y)[:, free]
        H = (gp - gm) / (2.0 * hstep[:, None])
        H = 0.5 * (H + H.T)
        W = np.zeros((nw, nw))
        W[:nf, :nf] = H
        with np.errstate(divide="ignore", invalid="ignore"):
            Sig = np.where(hasL, zL / (w - wl), 0.0) + np.where(hasU, zU / (wu - w), 0.0)
            gphi = gradw - np.where(hasL, mu / (w - wl), 0.0) + np.where(hasU, mu / (wu - w), 0.0)
        rhs = -np.concatenate([gphi + A.T @ y, c])
        # ---- inertia-corrected factorisation
        delta_w, delta_c = 0.0, 0.0
        for attempt in range(60):
            K = np.zeros((nw + m, nw + m))
            K[:nw, :nw] = W + np.diag(Sig + delta_w)
            K[:nw, nw:] = A.T
            K[nw:, :nw] = A
            K[nw:, nw:] = -delta_c * np.eye(m)
            lu, D, perm = ldl(K, lower=True)
            pos, neg, zero = _inertia(D, tol=1e-13 * max(1.0, np.abs(D).max()))
            if pos == nw and neg == m and zero == 0:
                break
            if zero > 0 and delta_c == 0.0:
                delta_c = 1e-8 * mu ** 0.25
                continue
            if delta_w == 0.0:
                delta_w = 1e-4 if delta_w_last == 0.0 else max(1e-20, delta_w_last / 3.0)
            else:
                delta_w *= 8.0 if delta_w_last else 100.0
        delta_w_last = delta_w
        sol = np.linalg.solve(K, rhs)
        dw, dy = sol[:nw], sol[nw:]
        if delta_c > 0.0:
            # rank-deficient constraints: keep the multipliers min-norm (drop their component in
            # null(A^T), which the regularised system inflates by ~1/delta_c and which changes
            # neither the Lagrangian gradient nor the step)
            U, sv, _ = np.linalg.svd(A, full_matrices=True)
            null = U[:, sv.size:] if sv.size < m else U[:, sv <= 1e-10 * max(sv.max(initial=0.0), 1.0)]
            if null.size:
                yn = y + dy
                dy = dy - null @ (null.T @ yn)
        with np.errstate(divide="ignore", invalid="ignore"):
            dzL = np.where(hasL, mu / (w - wl) - zL - zL / (w - wl) * dw, 0.0)
            dzU = np.where(hasU, mu / (wu - w) - zU + zU / (wu - w) * dw, 0.0)
        # ---- fraction to the boundary
        tau = tau_min

        def max_step(v, dv, lo_mask, lo):
            with np.errstate(divide="ignore", invalid="ignore"):
                r = np.where(lo_mask & (dv < 0), -tau * (v - lo) / dv, np.inf)
            return min(1.0, r.min(initial=np.inf))

        a_max = min(max_step(w, dw, hasL, wl), max_step(-w, -dw, hasU, -wu))
        a_z = min(max_step(zL, dzL, hasL, 0.0), max_step(zU, dzU, hasU, 0.0))
        # ---- backtracking on the l1 merit
        nu = max(nu, 1.1 * np.abs(y + dy).max(initial=0.0) + 1.0)
        phi0 = barrier_obj(f, w, mu) + nu * np.abs(c).sum()
        dphi = gphi @ dw - nu * np.abs(c).sum()
        alpha = a_max
        accepted = False
        for _ in range(40):
            wt = w + alpha * dw
            xt, st = unpack(wt)
            o = evals(xt)
            ct = cons(o["g"][0], st)
            phit = barrier_obj(o["f"][0], wt, mu) + nu * np.abs(ct).sum()
            if np.isfinite(phit) and phit <= phi0 + 1e-8 * alpha * min(dphi, 0.0):
                accepted = True
                break
            alpha *= 0.5
        if not accepted:
            alpha = a_max * 0.5 ** 10
        if verbose > 1:
            print(f"    alpha={alpha:.3e} a_max={a_max:.3e} a_z={a_z:.3e} phi0={phi0:.6e} dphi={dphi:.3e} "
                  f"|dw|={np.abs(dw).max():.2e} delta_w={delta_w:.1e} delta_c={delta_c:.1e}")
        w = w + alpha * dw
        y = y + alpha * dy
        zL = np.where(hasL, zL + a_z * dzL, 0.0)
        zU = np.where(hasU, zU + a_z * dzU, 0.0)
        # keep z within kappa_Sigma of mu / slack (IPOPT 1e10)
        with np.errstate(divide="ignore", invalid="ignore"):
            zL = np.where(hasL, np.clip(zL, mu / (1e10 * (w - wl)), 1e10 * mu / (w - wl)), 0.0)
            zU = np.where(hasU, np.clip(zU, mu / (1e10 * (wu - w)), 1e10 * mu / (wu - w)), 0.0)

    xx, s = unpack(w)
    problem.SetVariables(xx)
    o = evals(xx)
    c = cons(o["g"][0], s)
    dual = np.concatenate([o["grad"][0][free], np.zeros(nI)]) + jac_w(dense_J(o["jac"][0])).T @ y - zL + zU
    return IpmResult(x=xx, y=y, success=status == "optimal", status=status, iterations=it,
                     primal_inf=float(np.abs(c).max(initial=0.0)), dual_inf=float(np.abs(dual).max(initial=0.0)),
                     objective=float(o["f"][0]))
