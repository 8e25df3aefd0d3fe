"""Batched solve loop (BASELINE.json configs[4]): many concurrent
CentroidalPlanner solves driven in lock-step, every callback of every instance in ONE launch.

The reference solves one problem at a time with IPOPT through IFOPT's IpoptSolver
(src/CentroidalPlanner.cpp:22-34; IFOPT's defaults: exact constraint Jacobian, limited-memory
quasi-Newton Hessian, tol 1e-8).  IPOPT is not in this image and its MUMPS back end is not
re-entrant, so 8,192 concurrent IPOPT instances are not an option either.  This module restates
the parts of IPOPT's primal-dual interior-point method (Waechter & Biegler 2006) this problem class
uses, batched over instances, with every per-instance quantity a row of a device tensor:

  * variables w = [x_free, s]: fixed variables (x_l == x_u, CoMPlanner's positions / normals) are
    parameters (fixed_variable_treatment = make_parameter); one slack per inequality row
    (g_I(x) - s = 0, s within [g_l, g_u]); bound_push / bound_frac = 1e-2; bound multipliers start
    at 1 (bound_mult_init_val), constraint multipliers at the least-squares estimate when it is
    <= 1e3 (constr_mult_init_max);
  * Hessian of the Lagrangian (hessian="exact", IPOPT's default): central differences of its
    exact gradient grad f + J^T y over x_free, the 2 n_free perturbed points of every instance
    evaluated as ONE batch of B * 2 n_free instances; or (hessian="limited-memory", what IFOPT
    configures) a dense damped BFGS model initialised like IPOPT's scalar1 = s'y / s's;
  * Newton step by the null-space method in projector form, batched Cholesky factorisations only
    (A = [J_free | -P], G = A A^T, projector P = I - A^T G^-1 A onto null(A)): the KKT matrix
    has IPOPT's inertia (nw+, m-, 0) iff A has full row rank and the reduced Hessian
    Z^T (W + Sigma) Z is positive definite, i.e. iff P (W + Sigma) P + gamma (I - P) is, so that
    Cholesky's per-instance info is the inertia test (failure -> delta_w with IPOPT's schedule);
    a rank-deficient A (the single-contact torque about the force line) gets delta_c on G; one step
    of iterative refinement on the full KKT residual;
  * fraction-to-the-boundary rule (tau = max(0.99, 1 - mu)), monotone Fiacco-McCormick barrier
    update (kappa_mu = 0.2, theta_mu = 1.5, kappa_eps = 10) with a filter reset, IPOPT's filter
    line search (switching condition, Armijo on the barrier objective for f-type steps, filter
    augmentation after h-type steps) with up to four second-order corrections on the first trial,
    kappa_Sigma = 1e10 safeguard on the bound multipliers; no restoration phase: an instance whose
    line search finds no acceptable point takes the last trial and restarts its filter;
  * termination on IPOPT's scaled optimality error (s_max = 100) <= tol, or <= acceptable_tol
    (1e-6) for 15 consecutive iterations.

Every evaluation — the iterate and each line-search trial point — is ONE batched call of the
evaluator for all instances.  The product evaluator (KernelEvaluator) is the gfx950 eval kernel
through cpl_eval_batch on device-resident tensors (no host round trip); instances that converged
stay in the batch (frozen), so the launch shape never changes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import ctypes

import numpy as np

from . import _abi
from ._abi import INF

BIG = INF / 10.0  # |bound| >= 1e19 is infinite (IPOPT nlp_lower/upper_bound_inf)

STATUS_OPTIMAL = 0
STATUS_ACCEPTABLE = 1
STATUS_MAX_ITER = 2
STATUS_NAMES = {STATUS_OPTIMAL: "optimal", STATUS_ACCEPTABLE: "acceptable", STATUS_MAX_ITER: "max_iter"}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class KernelEvaluator:
    """The product callbacks: eval_f / eval_grad_f / eval_g / eval_jac_g of every instance in one
    cpl_eval_batch launch on device-resident tensors (CplProblem.eval_batch raises unless the
    inputs are CUDA tensors and the HIP library is loaded — there is no CPU fallback)."""

    def __init__(self, problem, env_tag=None):
        self.problem = problem
        self.env_tag = env_tag
        self.launches = 0
        self.instances = 0

    def __call__(self, X, mass):
        out = self.problem.eval_batch(X, mass, self.env_tag, outputs=("g", "jac", "f", "grad"))
        self.launches += 1
        self.instances += X.shape[0]
        return out


@dataclass
class BatchSolveResult:
    x: object            # [B, n] final iterates
    y: object            # [B, m] constraint multipliers
    status: object       # [B] int: STATUS_*
    iterations: object   # [B] iterations to termination
    objective: object    # [B]
    primal_inf: object   # [B] max constraint violation (unscaled, against g_l / g_u)
    dual_inf: object     # [B] max |grad_w L|
    evaluations: int     # evaluator calls (= launches with KernelEvaluator)
    iterations_run: int  # lock-step iterations of the batch

    @property
    def success(self):
        return self.status <= STATUS_ACCEPTABLE


def batch_ipm_solve(problem, X0, mass=None, evaluator: Optional[Callable] = None, tol: float = 1e-8,
                    max_iter: int = 3000, mu_init: float = 0.1, acceptable_tol: float = 1e-6,
                    acceptable_iter: int = 15, max_ls: int = 30, max_soc: int = 4, hessian: str = "exact",
                    fd_step: float = 1e-6, verbose: int = 0) -> BatchSolveResult:
    """Solve B instances of `problem`'s template from the starting points X0 [B, n] (torch float64,
    device tensor), per-instance robot masses `mass` [B] (None: the template's).

    evaluator(X [B, n], mass) -> {"f": [B], "grad": [B, n], "g": [B, m], "jac": [B, nnz]} on X's
    device; default KernelEvaluator(problem) (the HIP kernel).

    hessian: "exact" — the Hessian of the Lagrangian over x_free by central differences of its exact
    gradient grad f + J^T y, the 2 n_free perturbed points of every instance evaluated as ONE batch
    of B * 2 n_free instances (IPOPT's default hessian_approximation); "limited-memory" — the damped
    BFGS model (what IFOPT configures)."""
    if hessian not in ("exact", "limited-memory"):
        raise ValueError("hessian must be 'exact' or 'limited-memory'")
    use_bfgs = hessian == "limited-memory"
    import torch

    ev = evaluator if evaluator is not None else KernelEvaluator(problem)
    dev, dt = X0.device, torch.float64
    B = X0.shape[0]
    n, m, nnz = problem.get_nlp_info()
    iRow, jCol = problem.get_structure()
    xl_np, xu_np, gl_np, gu_np = problem.get_bounds_info()

    def T(a):
        return torch.as_tensor(np.asarray(a), dtype=dt, device=dev)

    xl, xu, gl, gu = T(xl_np), T(xu_np), T(gl_np), T(gu_np)
    flat_idx = torch.as_tensor(iRow.astype(np.int64) * n + jCol.astype(np.int64), device=dev)
    iRow_t = torch.as_tensor(iRow.astype(np.int64), device=dev)
    jCol_t = torch.as_tensor(jCol.astype(np.int64), device=dev)

    fixed_np = np.abs(xu_np - xl_np) <= 1e-14 * np.maximum(1.0, np.abs(xl_np))
    fixed = torch.as_tensor(np.where(fixed_np)[0], device=dev)
    free = torch.as_tensor(np.where(~fixed_np)[0], device=dev)
    nf = int((~fixed_np).sum())
    I_np = np.where(gl_np != gu_np)[0]
    I = torch.as_tensor(I_np, device=dev)
    nI = I_np.size
    nw = nf + nI
    zeros_B = torch.zeros(B, dtype=dt, device=dev)
    # A = dc/dw = [J[:, free] | -P], P[r, j] = 1 where row r is inequality j
    P = torch.zeros(m, nI, dtype=dt, device=dev)
    P[I, torch.arange(nI, device=dev)] = 1.0

    ninf = torch.full((nI,), -float("inf"), dtype=dt, device=dev)
    wl = torch.cat([xl[free], torch.where(gl[I] > -BIG, gl[I], ninf)])
    wu = torch.cat([xu[free], torch.where(gu[I] < BIG, gu[I], -ninf)])
    hasL, hasU = torch.isfinite(wl), torch.isfinite(wu)
    wl0, wu0 = torch.where(hasL, wl, torch.zeros_like(wl)), torch.where(hasU, wu, torch.zeros_like(wu))
    nbounds = int(hasL.sum().item() + hasU.sum().item())

    def push(v):  # IPOPT bound_push = bound_frac = 1e-2 (absolute and relative to the range)
        k = 1e-2
        rng = torch.where(hasL & hasU, wu0 - wl0, torch.full_like(wl0, float("inf")))
        pl = torch.minimum(k * torch.clamp(wl0.abs(), min=1.0), k * rng)
        pu = torch.minimum(k * torch.clamp(wu0.abs(), min=1.0), k * rng)
        v = torch.where(hasL, torch.maximum(v, wl0 + pl), v)
        return torch.where(hasU, torch.minimum(v, wu0 - pu), v)

    X = X0.to(dt).clone().contiguous()
    X[:, fixed] = xl[fixed]
    Mass = None if mass is None else mass.to(dt).contiguous()
    n_eval = 0

    def evaluate(Xe):
        nonlocal n_eval
        n_eval += 1
        o = ev(Xe, Mass)
        J = torch.zeros(B, m * n, dtype=dt, device=dev)
        J[:, flat_idx] = torch.nan_to_num(o["jac"], nan=0.0)  # a cone at F_t = 0 has a 0/0 Jacobian
        return {"f": o["f"].clone(), "grad": o["grad"].clone(), "g": o["g"].clone(), "J": J.view(B, m, n)}

    def unpack(wv):
        Xn = X.clone()
        Xn[:, free] = wv[:, :nf]
        return Xn.contiguous()

    def cons(g, s):
        c = g - gl
        c[:, I] = g[:, I] - s
        return c

    def jac_w(J):
        return torch.cat([J[:, :, free], (-P).expand(B, m, nI)], dim=2)

    def barrier(wv, muv):
        dl_ = torch.where(hasL, wv - wl0, torch.ones_like(wv))
        du_ = torch.where(hasU, wu0 - wv, torch.ones_like(wv))
        return -muv * (torch.log(dl_).sum(1) + torch.log(du_).sum(1))

    def lagrangian_grad(grad, jac, yv):  # grad f + J^T y from the CSR values
        out = grad.clone()
        out.index_add_(1, jCol_t, torch.nan_to_num(jac, nan=0.0) * yv[:, iRow_t])
        return out

    def fd_hessian(Xc, yv):
        nonlocal n_eval
        h = fd_step * torch.clamp(Xc[:, free].abs(), min=1.0)                       # [B, nf]
        Xp = Xc.unsqueeze(1).repeat(1, 2 * nf, 1)                                   # [B, 2nf, n]
        j = torch.arange(nf, device=dev)
        Xp[:, j, free] += h
        Xp[:, nf + j, free] -= h
        mp = None if Mass is None else Mass.repeat_interleave(2 * nf)
        n_eval += 1
        o = ev(Xp.view(B * 2 * nf, n).contiguous(), mp)
        gL = lagrangian_grad(o["grad"], o["jac"], yv.repeat_interleave(2 * nf, 0)).view(B, 2 * nf, n)[:, :, free]
        H = (gL[:, :nf] - gL[:, nf:]) / (2.0 * h[:, :, None])
        return 0.5 * (H + H.transpose(1, 2))

    # starting point: x pushed into its bounds, slacks = g_I(x) pushed into theirs
    X = unpack(push(torch.cat([X[:, free], torch.zeros(B, nI, dtype=dt, device=dev)], 1)))
    cur = evaluate(X)
    w = push(torch.cat([X[:, free], cur["g"][:, I]], 1))

    mu = torch.full((B,), mu_init, dtype=dt, device=dev)
    zL = torch.where(hasL, torch.ones_like(w), torch.zeros_like(w))
    zU = torch.where(hasU, torch.ones_like(w), torch.zeros_like(w))
    eye_m = torch.eye(m, dtype=dt, device=dev)
    eye_w = torch.eye(nw, dtype=dt, device=dev)
    eye_f = torch.eye(nf, dtype=dt, device=dev)
    Hq = eye_f.repeat(B, 1, 1)  # quasi-Newton Hessian of the Lagrangian over x_free
    hq_init = torch.zeros(B, dtype=torch.bool, device=dev)
    FMAX = 64
    filt_t = torch.full((B, FMAX), float("inf"), dtype=dt, device=dev)
    filt_p = torch.full((B, FMAX), float("inf"), dtype=dt, device=dev)
    fcount = torch.zeros(B, dtype=torch.int64, device=dev)
    theta0 = cons(cur["g"], w[:, nf:]).abs().sum(1)
    theta_max = 1e4 * theta0.clamp(min=1.0)
    theta_min = 1e-4 * theta0.clamp(min=1.0)

    def reset_filter(mask, ft, fp, fc):
        return (torch.where(mask[:, None], torch.full_like(ft, float("inf")), ft),
                torch.where(mask[:, None], torch.full_like(fp, float("inf")), fp),
                torch.where(mask, torch.zeros_like(fc), fc))

    delta_w_last = zeros_B.clone()
    use_hip = X0.is_cuda  # device tensors: the Newton step runs in cpl_kkt_solve
    if use_hip:
        kkt_ws = torch.empty(B * int(_abi.lib.cpl_kkt_workspace_doubles(nw, m)), dtype=dt, device=dev)

    # least-squares constraint multipliers (IPOPT constr_mult_init_max = 1e3)
    A = jac_w(cur["J"])
    gradw = torch.cat([cur["grad"][:, free], torch.zeros(B, nI, dtype=dt, device=dev)], 1)
    L0, info0 = torch.linalg.cholesky_ex(A @ A.transpose(1, 2) + 1e-12 * eye_m)
    y = -torch.cholesky_solve(A @ (gradw - zL + zU).unsqueeze(2), L0).squeeze(2)
    y = torch.where(((y.abs().amax(1) <= 1e3) & (info0 == 0)).unsqueeze(1), y, torch.zeros_like(y))

    active = torch.ones(B, dtype=torch.bool, device=dev)
    status = torch.full((B,), STATUS_MAX_ITER, dtype=torch.int64, device=dev)
    iters = torch.zeros(B, dtype=torch.int64, device=dev)
    acc_count = torch.zeros(B, dtype=torch.int64, device=dev)
    it_run = 0

    def errors(o, wv, yv, zl, zu, muv):
        A_ = jac_w(o["J"])
        gw = torch.cat([o["grad"][:, free], torch.zeros(B, nI, dtype=dt, device=dev)], 1)
        c_ = cons(o["g"], wv[:, nf:])
        dual = gw + (A_.transpose(1, 2) @ yv.unsqueeze(2)).squeeze(2) - zl + zu
        cl = torch.where(hasL, (wv - wl0) * zl, torch.zeros_like(wv))
        cu = torch.where(hasU, (wu0 - wv) * zu, torch.zeros_like(wv))
        s_max = 100.0
        zsum = zl.abs().sum(1) + zu.abs().sum(1)
        sd = torch.clamp((yv.abs().sum(1) + zsum) / max(m + nbounds, 1), min=s_max) / s_max
        sc = torch.clamp(zsum / max(nbounds, 1), min=s_max) / s_max
        d_inf_ = dual.abs().amax(1)
        c_inf = c_.abs().amax(1) if m else zeros_B
        comp = torch.maximum(cl.amax(1), cu.amax(1))
        comp_mu = torch.maximum((cl - torch.where(hasL, muv[:, None], 0.0)).abs().amax(1),
                                (cu - torch.where(hasU, muv[:, None], 0.0)).abs().amax(1))
        err0_ = torch.maximum(torch.maximum(d_inf_ / sd, c_inf), comp / sc)
        errmu_ = torch.maximum(torch.maximum(d_inf_ / sd, c_inf), comp_mu / sc)
        return A_, gw, c_, err0_, errmu_, d_inf_

    for it in range(max_iter + 1):
        A, gradw, c, err0, errmu, d_inf = errors(cur, w, y, zL, zU, mu)
        was_active = active
        done_now = active & (err0 <= tol)
        status = torch.where(done_now, torch.full_like(status, STATUS_OPTIMAL), status)
        acc_count = torch.where(active & (err0 <= acceptable_tol), acc_count + 1, torch.zeros_like(acc_count))
        acc_now = active & ~done_now & (acc_count >= acceptable_iter)
        status = torch.where(acc_now, torch.full_like(status, STATUS_ACCEPTABLE), status)
        active = active & ~done_now & ~acc_now
        iters = torch.where(was_active, torch.full_like(iters, it), iters)
        n_active = int(active.sum().item())
        if verbose:
            e = float(err0[active].max()) if n_active else 0.0
            print(f"it {it:4d} active {n_active:6d} max err0 {e:.3e}")
        if n_active == 0 or it == max_iter:
            break
        it_run = it + 1
        # ---- monotone barrier update (a few rounds, per instance)
        for _ in range(4):
            upd = active & (errmu <= 10.0 * mu) & (mu > tol / 10.0)
            if not bool(upd.any()):
                break
            mu = torch.where(upd, torch.clamp(torch.minimum(0.2 * mu, mu ** 1.5), min=tol / 10.0), mu)
            filt_t, filt_p, fcount = reset_filter(upd, filt_t, filt_p, fcount)
            errmu = errors(cur, w, y, zL, zU, mu)[4]
        tau = torch.clamp(1.0 - mu, min=0.99)

        dl = torch.where(hasL, w - wl0, torch.ones_like(w))
        du = torch.where(hasU, wu0 - w, torch.ones_like(w))
        Sig = torch.where(hasL, zL / dl, torch.zeros_like(w)) + torch.where(hasU, zU / du, torch.zeros_like(w))
        gphi = gradw - torch.where(hasL, mu[:, None] / dl, torch.zeros_like(w)) + \
            torch.where(hasU, mu[:, None] / du, torch.zeros_like(w))
        r1 = -(gphi + (A.transpose(1, 2) @ y.unsqueeze(2)).squeeze(2))
        r2 = -c
        M = torch.diag_embed(Sig)
        M[:, :nf, :nf] += Hq if use_bfgs else fd_hessian(X, y)
        if use_hip:
            # ---- Newton step on the device: cpl_kkt_solve (csrc/cpl_kkt.hip) — null-space method
            # on a Householder QR of A^T, IPOPT's inertia correction and one refinement step, one
            # workgroup per instance, no host synchronisation
            Mc, Ac = M.contiguous(), A.contiguous()
            r1c = r1.contiguous()
            act_u8 = active.to(torch.uint8)
            kkt_dw = torch.empty(B, nw, dtype=dt, device=dev)
            kkt_dy = torch.empty(B, m, dtype=dt, device=dev)
            delta_w = torch.empty(B, dtype=dt, device=dev)
            delta_c = torch.empty(B, dtype=dt, device=dev)
            kkt_info = torch.empty(B, dtype=torch.int32, device=dev)
            stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            _abi.check(_abi.lib.cpl_kkt_solve(0, B, nw, m, _ptr(Mc), _ptr(Ac), _ptr(r1c), _ptr(r2.contiguous()),
                                              _ptr(mu.contiguous()), _ptr(delta_w_last.contiguous()), _ptr(act_u8),
                                              _ptr(kkt_dw), _ptr(kkt_dy), _ptr(delta_w), _ptr(delta_c),
                                              _ptr(kkt_info), _ptr(kkt_ws), stream))
            delta_w_last = torch.where(active, delta_w, delta_w_last)
            dw, dy = kkt_dw, kkt_dy

            def solve_primal(r2v):  # second-order correction: the kept factors, another r2
                out_dw = torch.empty(B, nw, dtype=dt, device=dev)
                out_dy = torch.empty(B, m, dtype=dt, device=dev)
                _abi.check(_abi.lib.cpl_kkt_solve(1, B, nw, m, _ptr(Mc), _ptr(Ac), _ptr(r1c), _ptr(r2v.contiguous()),
                                                  None, None, _ptr(act_u8), _ptr(out_dw), _ptr(out_dy), None, None,
                                                  None, _ptr(kkt_ws), stream))
                return out_dw
        else:
            # host tensors (the solver's logic under test on the CPU, with the oracle's callbacks):
            # the same Newton step with torch's dense factorisations
            # ---- Newton step, null-space method in projector form (batched Cholesky only):
            #   G = A A^T (+ delta_c I where A is rank-deficient), P = I - A^T G^-1 A (projector on
            #   null(A)), gamma > 0:
            #   min-norm part    dw_y = A^T G^-1 r2
            #   null-space part  (P M P + gamma (I - P)) v = P (r1 - M dw_y),   dw = dw_y + v
            #   multipliers      G dy = A (r1 - M dw)
            # In a basis [Z Y] the matrix P M P + gamma (I - P) is Z^T M Z (+) gamma I, so it is positive
            # definite iff the reduced Hessian is: the KKT matrix has IPOPT's inertia (nw+, m-, 0) iff
            # this Cholesky succeeds (failure -> delta_w on M, IPOPT's schedule), and v stays in null(A).
            # One step of iterative refinement on the full KKT residual follows.
            G = A @ A.transpose(1, 2)
            LG, infoG = torch.linalg.cholesky_ex(G)
            delta_c = zeros_B.clone()
            for _ in range(12):
                bad = infoG != 0
                if not bool(bad.any()):
                    break
                gscale = G.diagonal(dim1=1, dim2=2).amax(1).clamp(min=1e-300)
                delta_c = torch.where(bad, torch.where(delta_c == 0, 1e-8 * mu ** 0.25 * gscale, delta_c * 100.0), delta_c)
                LGn, infoGn = torch.linalg.cholesky_ex(G + delta_c[:, None, None] * eye_m)
                LG = torch.where(bad[:, None, None], LGn, LG)
                infoG = torch.where(bad, infoGn, infoG)
            GiA = torch.cholesky_solve(A, LG)                                   # [B, m, nw]
            Pn = eye_w - A.transpose(1, 2) @ GiA                                # [B, nw, nw]
            gamma = M.diagonal(dim1=1, dim2=2).abs().mean(1).clamp(min=1.0)
            PMP = Pn @ M @ Pn
            Kp = PMP + gamma[:, None, None] * (eye_w - Pn)
            delta_w = zeros_B.clone()
            L1, info1 = torch.linalg.cholesky_ex(Kp)
            for _ in range(40):
                bad = info1 != 0
                if not bool(bad.any()):
                    break
                first_dw = torch.where(delta_w_last == 0, torch.full_like(delta_w, 1e-4),
                                       torch.clamp(delta_w_last / 3.0, min=1e-20))
                grow = delta_w * torch.where(delta_w_last == 0, 100.0, 8.0)
                delta_w = torch.where(bad, torch.where(delta_w == 0, first_dw, grow), delta_w)
                L1n, info1n = torch.linalg.cholesky_ex(Kp + delta_w[:, None, None] * Pn)
                L1 = torch.where(bad[:, None, None], L1n, L1)
                info1 = torch.where(bad, info1n, info1)
            delta_w_last = torch.where(active, delta_w, delta_w_last)
            Mw = M + delta_w[:, None, None] * eye_w

            def kkt_solve(q1, q2):
                dwy = (GiA.transpose(1, 2) @ q2.unsqueeze(2))                     # A^T G^-1 q2
                rv = Pn @ (q1.unsqueeze(2) - Mw @ dwy)
                dw_ = dwy + torch.cholesky_solve(rv, L1)
                dy_ = torch.cholesky_solve(A @ (q1.unsqueeze(2) - Mw @ dw_), LG)
                return dw_.squeeze(2), dy_.squeeze(2)

            def kkt_refined(q1, q2):
                d1, d2 = kkt_solve(q1, q2)
                e1 = q1 - (Mw @ d1.unsqueeze(2)).squeeze(2) - (A.transpose(1, 2) @ d2.unsqueeze(2)).squeeze(2)
                e2 = q2 - (A @ d1.unsqueeze(2)).squeeze(2) + delta_c[:, None] * d2
                c1, c2 = kkt_solve(e1, e2)
                return d1 + c1, d2 + c2

            dw, dy = kkt_refined(r1, r2)

            def solve_primal(r2v):  # the same factorisations, another constraint right-hand side (SOC)
                return kkt_refined(r1, r2v)[0]
        dzL = torch.where(hasL, mu[:, None] / dl - zL - zL / dl * dw, torch.zeros_like(w))
        dzU = torch.where(hasU, mu[:, None] / du - zU + zU / du * dw, torch.zeros_like(w))

        # ---- fraction to the boundary
        def max_step(v, dv, lo_mask, lo):
            r = torch.where(lo_mask & (dv < 0), -tau[:, None] * (v - lo) / torch.where(dv < 0, dv, -1.0),
                            torch.full_like(v, float("inf")))
            return torch.clamp(r.amin(1), max=1.0)

        a_max = torch.minimum(max_step(w, dw, hasL, wl0), max_step(-w, -dw, hasU, -wu0))
        a_z = torch.minimum(max_step(zL, dzL, hasL, 0.0), max_step(zU, dzU, hasU, 0.0))

        # ---- filter line search (IPOPT: gamma_theta 1e-5, gamma_phi 1e-8, delta 1, s_theta 1.1,
        # s_phi 2.3, eta_phi 1e-8, theta_min/max = 1e-4/1e4 max(1, theta_0)) with up to max_soc
        # second-order corrections on the first trial; every trial point of every instance is one
        # batched evaluation
        theta_k = c.abs().sum(1)
        phi_k = cur["f"] + barrier(w, mu)
        gd = (gphi * dw).sum(1)
        switch_ok = (theta_k <= theta_min) & (gd < 0)
        alpha = a_max.clone()
        searching = active.clone()
        new = dict(cur)
        w_new = w
        accepted = torch.zeros(B, dtype=torch.bool, device=dev)
        aug = torch.zeros(B, dtype=torch.bool, device=dev)

        def judge(wt, o, al):
            ct = cons(o["g"], wt[:, nf:])
            th = ct.abs().sum(1)
            ph = o["f"] + barrier(wt, mu)
            fin = torch.isfinite(ph) & torch.isfinite(th)
            in_filter = ((th[:, None] <= (1.0 - 1e-5) * filt_t) | (ph[:, None] <= filt_p - 1e-8 * filt_t)).all(1)
            ftype = switch_ok & (al * (-gd).clamp(min=0.0) ** 2.3 > theta_k ** 1.1)
            armijo = ph <= phi_k + 1e-8 * al * gd
            suff = (th <= (1.0 - 1e-5) * theta_k) | (ph <= phi_k - 1e-8 * theta_k)
            ok = fin & (th <= theta_max) & in_filter & torch.where(ftype, armijo, suff)
            return ok, ~(ftype & armijo), th

        def take(mask, wt, o, aug_mask):
            nonlocal w_new, new, accepted, aug, searching
            for k in new:
                new[k] = torch.where(mask.view(-1, *([1] * (new[k].dim() - 1))), o[k], new[k])
            w_new = torch.where(mask[:, None], wt, w_new)
            aug = torch.where(mask, aug_mask, aug)
            accepted = accepted | mask
            searching = searching & ~mask

        for ls in range(max_ls):
            wt = w + alpha[:, None] * dw
            o = evaluate(unpack(torch.where(searching[:, None], wt, w_new)))
            ok, augm, th = judge(wt, o, alpha)
            take(searching & ok, wt, o, augm)
            if ls == 0 and max_soc > 0:
                # second-order corrections where the full trial step increased the infeasibility
                soc = searching & (th >= theta_k)
                c_soc = c.clone()
                a_soc = alpha.clone()
                th_old = theta_k.clone()
                ct = cons(o["g"], wt[:, nf:])
                for _ in range(max_soc):
                    if not bool(soc.any()):
                        break
                    c_soc = a_soc[:, None] * c_soc + ct
                    dws = solve_primal(-c_soc)
                    a_soc = torch.minimum(max_step(w, dws, hasL, wl0), max_step(-w, -dws, hasU, -wu0))
                    ws = w + a_soc[:, None] * dws
                    os_ = evaluate(unpack(torch.where(soc[:, None], ws, w_new)))
                    oks, augs, ths = judge(ws, os_, alpha)
                    take(soc & oks, ws, os_, augs)
                    soc = soc & ~oks & (ths <= 0.99 * th_old)  # kappa_soc = 0.99
                    th_old = ths
                    ct = cons(os_["g"], ws[:, nf:])
            if not bool(searching.any()):
                break
            alpha = torch.where(searching, 0.5 * alpha, alpha)
        # no acceptable trial (IPOPT would enter its restoration phase): take the last trial point and
        # restart that instance's filter
        failed = searching.clone()
        if bool(failed.any()):
            take(failed, wt, o, torch.zeros_like(failed))
        # augment the filter after h-type iterations, reset it where the line search failed
        slot = torch.remainder(fcount, FMAX)
        addm = aug & active
        fi = torch.arange(FMAX, device=dev)[None, :] == slot[:, None]
        filt_t = torch.where(addm[:, None] & fi, ((1.0 - 1e-5) * theta_k)[:, None], filt_t)
        filt_p = torch.where(addm[:, None] & fi, (phi_k - 1e-8 * theta_k)[:, None], filt_p)
        fcount = fcount + addm.to(fcount.dtype)
        filt_t, filt_p, fcount = reset_filter(failed, filt_t, filt_p, fcount)

        if verbose > 1:
            b = int(verbose) - 2
            print(f"   [{b}] mu={float(mu[b]):.2e} err0={float(err0[b]):.2e} dinf={float(d_inf[b]):.2e} cinf={float(c[b].abs().max()):.2e} "
                  f"a_max={float(a_max[b]):.2e} alpha={float(alpha[b]):.2e} a_z={float(a_z[b]):.2e} dw={float(dw[b].abs().max()):.2e} "
                  f"dy={float(dy[b].abs().max()):.2e} dW={float(delta_w[b]):.1e} dC={float(delta_c[b]):.1e} f={float(cur['f'][b]):.6e}")
        # ---- accept: primal, multipliers, bound multipliers (kappa_Sigma safeguard)
        act = active[:, None]
        y_new = torch.where(act, y + alpha[:, None] * dy, y)
        zL_new = torch.where(act & hasL, zL + a_z[:, None] * dzL, zL)
        zU_new = torch.where(act & hasU, zU + a_z[:, None] * dzU, zU)
        dln = torch.where(hasL, w_new - wl0, torch.ones_like(w))
        dun = torch.where(hasU, wu0 - w_new, torch.ones_like(w))
        zL_new = torch.where(act & hasL, torch.minimum(torch.maximum(zL_new, mu[:, None] / (1e10 * dln)),
                                                       1e10 * mu[:, None] / dln), zL_new)
        zU_new = torch.where(act & hasU, torch.minimum(torch.maximum(zU_new, mu[:, None] / (1e10 * dun)),
                                                       1e10 * mu[:, None] / dun), zU_new)

        # ---- damped BFGS update of the Lagrangian Hessian over x_free (both gradients at the new y)
        sk = (w_new - w)[:, :nf]
        JTy_new = (new["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
        JTy_old = (cur["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
        yk = (new["grad"] + JTy_new)[:, free] - (cur["grad"] + JTy_old)[:, free]
        sy = (sk * yk).sum(1)
        ss = (sk * sk).sum(1)
        first = use_bfgs & active & ~hq_init & (sy > 0) & (ss > 0)
        sigma0 = torch.where(first, sy / torch.where(ss > 0, ss, 1.0), torch.ones_like(sy))
        Hq = torch.where(first[:, None, None], sigma0[:, None, None] * eye_f, Hq)
        hq_init = hq_init | first
        Hs = (Hq @ sk.unsqueeze(2)).squeeze(2)
        sHs = (sk * Hs).sum(1)
        theta = torch.where(sy >= 0.2 * sHs, torch.ones_like(sy),
                            0.8 * sHs / torch.where(sHs - sy != 0, sHs - sy, 1.0))
        r = theta[:, None] * yk + (1.0 - theta[:, None]) * Hs
        sr = (sk * r).sum(1)
        upd = use_bfgs & active & (ss > 1e-30) & (sHs > 0) & (sr > 0)
        Hn = Hq - Hs.unsqueeze(2) * Hs.unsqueeze(1) / torch.where(upd, sHs, 1.0)[:, None, None] + \
            r.unsqueeze(2) * r.unsqueeze(1) / torch.where(upd, sr, 1.0)[:, None, None]
        Hq = torch.where(upd[:, None, None], 0.5 * (Hn + Hn.transpose(1, 2)), Hq)

        w = torch.where(act, w_new, w)
        y, zL, zU = y_new, zL_new, zU_new
        cur = {k: torch.where(active.view(-1, *([1] * (v.dim() - 1))), new[k], v) for k, v in cur.items()}
        X = unpack(w)

    g = cur["g"]
    viol = torch.clamp(torch.maximum(gl - g, g - gu), min=0.0).amax(1) if m else zeros_B
    return BatchSolveResult(x=X, y=y, status=status, iterations=iters, objective=cur["f"], primal_inf=viol,
                            dual_inf=d_inf, evaluations=n_eval, iterations_run=it_run)
