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
    (g_I(x) - s = 0, s within [g_l, g_u]); bounds relaxed by bound_relax_factor = 1e-8, the final
    point projected back (honor_original_bounds);
    bound_push / bound_frac = 1e-2; bound multipliers start
    at 1 (bound_mult_init_val), constraint multipliers at the least-squares estimate when it is
    <= 1e3 (constr_mult_init_max);
  * Hessian of the Lagrangian (hessian="exact", IPOPT's default): central differences of its
    exact gradient grad f + J^T y over x_free, the 2 n_free perturbed points of every instance
    evaluated as ONE batch of B * 2 n_free instances and J^T y formed on the device
    (cpl_lagrangian_grad); or (hessian="limited-memory", what IFOPT configures) a dense damped BFGS
    model initialised like IPOPT's scalar1 = s'y / s's;
  * Newton step (cpl_kkt_solve, csrc/cpl_kkt.hip): null-space method on a Householder QR of A^T
    (A = [J_free | -P]) with IPOPT's inertia correction on the device — the KKT matrix has inertia
    (nw+, m-, 0) iff A has full row rank and the reduced Hessian Z^T (W + Sigma) Z is positive
    definite, so its Cholesky is the inertia test (failure -> delta_w with IPOPT's schedule); a
    rank-deficient A (the single-contact torque about the force line) gets delta_c; one step of
    iterative refinement.  Host tensors (the solver's logic under test on the CPU) take the same
    step from torch's dense factorisations (projector form of the null-space method);
  * fraction-to-the-boundary rule (tau = max(0.99, 1 - mu)), monotone Fiacco-McCormick barrier
    update (kappa_mu = 0.2, theta_mu = 1.5, kappa_eps = 10) with a filter reset, IPOPT's filter
    line search (switching condition, Armijo on the barrier objective for f-type steps, filter
    augmentation after h-type steps) with second-order corrections on the first trial,
    kappa_Sigma = 1e10 safeguard on the bound multipliers; no restoration phase: an instance whose
    line search finds no acceptable point takes one feasibility (min-norm Gauss-Newton) step when
    that cuts its violation, else the last trial, and restarts its filter;
  * termination on IPOPT's scaled optimality error (s_max = 100) <= tol, or <= acceptable_tol
    (1e-6) for 15 consecutive iterations.

Every evaluation — the iterate, each line-search trial point, the finite-difference points — is ONE
batched call of the evaluator for all instances.  The product evaluator (KernelEvaluator) is the
gfx950 eval kernel through cpl_eval_batch on device-resident tensors.  Instances that converged
stay in the batch (frozen), so every launch keeps its shape; one iteration has no host
synchronisation at all (fixed trip counts, masked updates), and on the device it is captured once
as a HIP graph and replayed — on the device path the host reads an "any active" flag one iteration
behind (no stall); on host tensors it checks every `check_every` iterations whether any
instance is still active.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import _abi
from ._abi import INF

BIG = INF / 10.0  # |bound| >= 1e19 is infinite (IPOPT nlp_lower/upper_bound_inf)

STATUS_OPTIMAL = 0
STATUS_ACCEPTABLE = 1
STATUS_MAX_ITER = 2
STATUS_NAMES = {STATUS_OPTIMAL: "optimal", STATUS_ACCEPTABLE: "acceptable", STATUS_MAX_ITER: "max_iter"}

FMAX = 64  # filter entries kept per instance (a ring)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class KernelEvaluator:
    """The product callbacks: eval_f / eval_grad_f / eval_g / eval_jac_g of every instance in one
    cpl_eval_batch launch on device-resident tensors (CplProblem.eval_batch raises unless the
    inputs are CUDA tensors and the HIP library is loaded — there is no CPU fallback)."""

    def __init__(self, problem, env_tag=None):
        self.problem = problem
        self.env_tag = env_tag
        self.calls = 0

    def __call__(self, X, mass, outputs=("g", "jac", "f", "grad"), jac_folded=False):
        """jac_folded: values-only Jacobian records (CPL_EVAL_JAC_FOLDED; CplProblem.jac_fold_info)."""
        self.calls += 1
        return self.problem.eval_batch(X, mass, self.env_tag, outputs=outputs, jac_folded=jac_folded)

    def lagrangian_grad(self, X, mass, y, y_repeat, csc, active=None):
        """grad f + J^T y of every instance in one fused launch (cpl_eval_lagrangian_grad: the
        Jacobian stays in LDS); None where the fused path does not exist (Superquadric / mixed
        batches: the caller takes eval + cpl_lagrangian_grad, the same result)."""
        import torch

        if getattr(self, "_no_fused", False):
            return None
        out = torch.empty(X.shape[0], X.shape[1], dtype=torch.float64, device=X.device)
        st = _abi.lib.cpl_eval_lagrangian_grad(
            ctypes.byref(self.problem.desc()), X.shape[0], _ptr(X), None if mass is None else _ptr(mass),
            None if self.env_tag is None else _ptr(self.env_tag), _ptr(csc[0]), _ptr(csc[1]), _ptr(csc[2]), _ptr(y),
            y_repeat, None if active is None else _ptr(active), _ptr(out),
            ctypes.c_void_p(torch.cuda.current_stream(X.device).cuda_stream))
        if st == _abi.ERR_UNSUPPORTED:
            self._no_fused = True
            return None
        _abi.check(st)
        self.calls += 1
        return out


@dataclass
class BatchSolveResult:
    x: object            # [B, n] final iterates
    y: object            # [B, m] constraint multipliers
    status: object       # [B] int: STATUS_*
    iterations: object   # [B] Newton steps taken until termination
    objective: object    # [B]
    primal_inf: object   # [B] max constraint violation (unscaled, against g_l / g_u)
    dual_inf: object     # [B] max |grad_w L|
    evaluations: int     # batched evaluator launches (graph replays included)
    iterations_run: int  # lock-step iterations of the batch
    graph: bool          # the iteration ran as a captured HIP graph

    @property
    def success(self):
        return self.status <= STATUS_ACCEPTABLE


_PIVOT_REL = 2.220446049250313e-16  # DBL_EPSILON: the KKT inertia test's zero-pivot level


def batch_ipm_solve(problem, X0, mass=None, evaluator: Optional[Callable] = None, tol: float = 1e-8,
                    max_iter: int = 3000, mu_init: float = 0.1, acceptable_tol: float = 1e-6,
                    acceptable_iter: int = 15, max_ls: int = 4, max_soc: int = 1, hessian: str = "exact",
                    fd_step: float = 1e-6, graph: Optional[bool] = None, check_every: int = 4,
                    verbose: int = 0) -> BatchSolveResult:
    """Solve B instances of `problem`'s template from the starting points X0 [B, n] (torch float64,
    device tensor), per-instance robot masses `mass` [B] (None: the template's).

    evaluator(X [B, n], mass, outputs) -> {name: tensor} for outputs among "f" [B], "grad" [B, n],
    "g" [B, m], "jac" [B, nnz], on X's device; default KernelEvaluator(problem) (the HIP kernel).
    hessian: "exact" (the analytic Lagrangian Hessian, cpl_lagrangian_hessian, for Ground /
    no-environment problems on the device; batched central differences of the Lagrangian gradient
    otherwise), "fd" (always the central differences) or "limited-memory"
    (damped BFGS).  graph: capture one iteration as a HIP graph (default: on for device tensors).
    max_ls / max_soc: line-search trials / second-order corrections per iteration (fixed counts)."""
    if hessian not in ("exact", "fd", "limited-memory"):
        raise ValueError("hessian must be 'exact', 'fd' or 'limited-memory'")
    use_bfgs = hessian == "limited-memory"
    import torch

    ev = evaluator if evaluator is not None else KernelEvaluator(problem)
    dev, dt = X0.device, torch.float64
    use_hip = X0.is_cuda  # device tensors: Newton step and J^T y on the device
    use_graph = (use_hip if graph is None else bool(graph)) and verbose <= 1
    if use_graph and not use_hip:
        raise ValueError("graph capture needs device tensors")
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
    if use_hip and nw > 128:  # the device kernels stage one instance's primal-slack vector per wave
        raise ValueError(f"batch_ipm_solve: {nw} primal-slack unknowns (free variables + inequality rows); "
                         "the device solve loop supports at most 128 (about 11 contacts with an environment)")
    zeros_B = torch.zeros(B, dtype=dt, device=dev)
    # A = dc/dw = [J[:, free] | -P], P[r, j] = 1 where row r is inequality j
    P = torch.zeros(m, nI, dtype=dt, device=dev)
    P[I, torch.arange(nI, device=dev)] = 1.0
    zeros_I = torch.zeros(B, nI, dtype=dt, device=dev)

    ninf = torch.full((nI,), -float("inf"), dtype=dt, device=dev)
    wl = torch.cat([xl[free], torch.where(gl[I] > -BIG, gl[I], ninf)])
    wu = torch.cat([xu[free], torch.where(gu[I] < BIG, gu[I], -ninf)])
    # IPOPT bound_relax_factor = 1e-8: every finite bound moves outwards by 1e-8 max(1, |bound|), so
    # an inequality that is identically active (a lifting contact's cone rows at F = 0) keeps an
    # interior for its slack
    wl = wl - 1e-8 * torch.clamp(wl.abs(), min=1.0)
    wu = wu + 1e-8 * torch.clamp(wu.abs(), min=1.0)
    hasL, hasU = torch.isfinite(wl), torch.isfinite(wu)
    wl0, wu0 = torch.where(hasL, wl, torch.zeros_like(wl)), torch.where(hasU, wu, torch.zeros_like(wu))
    nbounds = int(hasL.sum().item() + hasU.sum().item())
    hasL_u8, hasU_u8 = hasL.to(torch.uint8).contiguous(), hasU.to(torch.uint8).contiguous()
    eye_m = torch.eye(m, dtype=dt, device=dev)
    eye_w = torch.eye(nw, dtype=dt, device=dev)
    eye_f = torch.eye(nf, dtype=dt, device=dev)
    fslot = torch.arange(FMAX, device=dev)[None, :]
    fd_cols = torch.arange(nf, device=dev)

    # transposed (CSC) index of the fixed CSR structure, for the device Lagrangian gradient
    order = np.lexsort((iRow, jCol))
    col_ptr_np = np.zeros(n + 1, dtype=np.int64)
    np.add.at(col_ptr_np, jCol.astype(np.int64) + 1, 1)
    col_ptr_np = np.cumsum(col_ptr_np)
    csc = [torch.as_tensor(a.astype(np.int32), device=dev) for a in (col_ptr_np, order, iRow[order])]
    row_slack_np = np.full(m, -1, dtype=np.int32)
    row_slack_np[I_np] = np.arange(nI, dtype=np.int32)
    row_slack = torch.as_tensor(row_slack_np, device=dev)
    # device path: the Jacobian state stays in CSR form; A = [J_free | -P] is gathered per iteration
    csr_J = use_hip and not use_bfgs
    dense_pos = np.full(m * n, -1, dtype=np.int64)
    dense_pos[iRow.astype(np.int64) * n + jCol.astype(np.int64)] = np.arange(nnz)
    # the product evaluator writes values-only Jacobian records (the structural constants skipped,
    # CPL_EVAL_JAC_FOLDED): amap points into the folded record, -2 marks a skipped constant 1
    folded = csr_J and isinstance(ev, KernelEvaluator)
    if folded:
        var_k, const_k, const_val = problem.jac_fold_info()
        rec_pos = np.full(nnz, -1, dtype=np.int64)
        rec_pos[var_k] = np.arange(var_k.size)
        rec_pos[const_k[const_val == 1.0]] = -2
        assert set(np.unique(const_val)) <= {0.0, 1.0}
        dense_rec = np.where(dense_pos >= 0, rec_pos[np.maximum(dense_pos, 0)], -1)
        nnz_rec = int(var_k.size)
    else:
        dense_rec, nnz_rec = dense_pos, nnz
    amap = torch.as_tensor(dense_rec.reshape(m, n)[:, np.where(~fixed_np)[0]].astype(np.int32).copy(), device=dev)
    if use_hip:
        kkt_ws = torch.empty(B * int(_abi.lib.cpl_kkt_workspace_doubles(nw, m)), dtype=dt, device=dev)

    def push(v):  # IPOPT bound_push = bound_frac = 1e-2 (absolute and relative to the range)
        k = 1e-2
        rng = torch.where(hasL & hasU, wu0 - wl0, torch.full_like(wl0, float("inf")))
        pl = torch.minimum(k * torch.clamp(wl0.abs(), min=1.0), k * rng)
        pu = torch.minimum(k * torch.clamp(wu0.abs(), min=1.0), k * rng)
        v = torch.where(hasL, torch.maximum(v, wl0 + pl), v)
        return torch.where(hasU, torch.minimum(v, wu0 - pu), v)

    Xbase = X0.to(dt).clone().contiguous()
    Xbase[:, fixed] = xl[fixed]
    Mass = None if mass is None else mass.to(dt).contiguous()
    Mass_fd = None if Mass is None else Mass.repeat_interleave(2 * nf).contiguous()
    n_eval = 0

    def stream():
        return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream) if use_hip else None

    def evaluate_fg(Xe):  # line-search trial points: constraint values and objective only
        nonlocal n_eval
        n_eval += 1
        o = ev(Xe, Mass, outputs=("g", "f"))
        return {"f": o["f"], "g": o["g"]}

    def evaluate(Xe):
        nonlocal n_eval
        n_eval += 1
        o = ev(Xe, Mass, jac_folded=True) if folded else ev(Xe, Mass)
        if csr_J:  # the device path keeps the Jacobian records; jac_w builds A from them in one launch
            return {"f": o["f"], "grad": o["grad"], "g": o["g"], "J": o["jac"].contiguous()}
        J = torch.zeros(B, m * n, dtype=dt, device=dev)
        J[:, flat_idx] = torch.nan_to_num(o["jac"], nan=0.0)  # a cone at F_t = 0 has a 0/0 Jacobian
        return {"f": o["f"], "grad": o["grad"], "g": o["g"], "J": J.view(B, m, n)}

    def unpack(wv):
        Xn = Xbase.clone()
        Xn[:, free] = wv[:, :nf]
        return Xn

    def cons(g, s):
        c = g - gl
        c[:, I] = g[:, I] - s
        return c

    def jac_w(J, mask=None):
        if csr_J:  # mask: rows of inactive instances are left unwritten (never read for them)
            A_ = torch.empty(B, m, nw, dtype=dt, device=dev)
            _abi.check(_abi.lib.cpl_ipm_dense_a(B, m, nw, nf, nnz_rec, _ptr(amap), _ptr(row_slack), _ptr(J), _ptr(A_),
                                                None if mask is None else _ptr(mask), stream()))
            return A_
        return torch.cat([J[:, :, free], (-P).expand(B, m, nI)], dim=2)

    def barrier(wv, muv):
        dl_ = torch.where(hasL, wv - wl0, torch.ones_like(wv))
        du_ = torch.where(hasU, wu0 - wv, torch.ones_like(wv))
        return -muv * (torch.log(dl_).sum(1) + torch.log(du_).sum(1))

    def fd_hessian(Xc, yv):
        nonlocal n_eval
        h = fd_step * torch.clamp(Xc[:, free].abs(), min=1.0)                       # [B, nf]
        Xp = Xc.unsqueeze(1).repeat(1, 2 * nf, 1)                                   # [B, 2nf, n]
        Xp[:, fd_cols, free] += h
        Xp[:, nf + fd_cols, free] -= h
        n_eval += 1
        fused = ev.lagrangian_grad if use_hip and hasattr(ev, "lagrangian_grad") else None
        gL = fused(Xp.view(B * 2 * nf, n), Mass_fd, yv.contiguous(), 2 * nf, csc) if fused else None
        if gL is not None:  # one launch: eval + grad f + J^T y from the LDS tile image
            pass
        elif use_hip:  # grad f + J^T y on the device (cpl_lagrangian_grad), y shared by the 2 nf points
            o = ev(Xp.view(B * 2 * nf, n), Mass_fd, outputs=("jac", "grad"))
            gL = torch.empty(B * 2 * nf, n, dtype=dt, device=dev)
            yc = yv.contiguous()
            _abi.check(_abi.lib.cpl_lagrangian_grad(B * 2 * nf, n, m, nnz, _ptr(csc[0]), _ptr(csc[1]), _ptr(csc[2]),
                                                    _ptr(o["grad"]), _ptr(o["jac"]), _ptr(yc), 2 * nf, _ptr(gL),
                                                    stream()))
        else:
            o = ev(Xp.view(B * 2 * nf, n), Mass_fd, outputs=("jac", "grad"))
            gL = o["grad"].clone()
            gL.index_add_(1, jCol_t, torch.nan_to_num(o["jac"], nan=0.0) * yv.repeat_interleave(2 * nf, 0)[:, iRow_t])
        gL = gL.view(B, 2 * nf, n)[:, :, free]
        H = (gL[:, :nf] - gL[:, nf:]) / (2.0 * h[:, :, None])
        return 0.5 * (H + H.transpose(1, 2))

    # the analytic Hessian kernel where the problem's environment allows it (a batch-0 call only
    # validates: CPL_ERR_UNSUPPORTED for Superquadric / mixed)
    analytic_H = (use_hip and hessian == "exact" and
                  _abi.lib.cpl_lagrangian_hessian(ctypes.byref(problem.desc()), 0, None, None, None, None, max(nf, 1),
                                                  None, None) == _abi.OK)
    free_i32 = torch.as_tensor(np.where(~fixed_np)[0].astype(np.int32), device=dev)
    Mr_buf = torch.zeros(B, nw, nw, dtype=dt, device=dev) if use_hip else None  # feasibility-step matrix
    freepos_np = np.full(n, -1, dtype=np.int32)
    freepos_np[np.where(~fixed_np)[0]] = np.arange(nf, dtype=np.int32)
    freepos = torch.as_tensor(freepos_np, device=dev)

    def fd_grads_dev(Xc, yv):
        """Device path of fd_hessian: the 2 nf points of every instance (cpl_ipm_fd_points) and their
        Lagrangian gradients (one fused eval launch); the differencing happens in the Newton setup."""
        nonlocal n_eval
        Xp = torch.empty(B * 2 * nf, n, dtype=dt, device=dev)
        h = torch.empty(B, nf, dtype=dt, device=dev)
        _abi.check(_abi.lib.cpl_ipm_fd_points(B, n, nf, fd_step, _ptr(freepos), _ptr(Xc.contiguous()), _ptr(Xp),
                                              _ptr(h), _ptr(S["active"]), stream()))
        n_eval += 1
        yc = yv.contiguous()
        fused = ev.lagrangian_grad if hasattr(ev, "lagrangian_grad") else None
        # converged instances are skipped: their rows of gL stay unwritten and only ever feed their
        # own (masked) Newton step
        gL = fused(Xp, Mass_fd, yc, 2 * nf, csc, S["active"]) if fused else None
        if gL is None:
            o = ev(Xp, Mass_fd, outputs=("jac", "grad"))
            gL = torch.empty(B * 2 * nf, n, dtype=dt, device=dev)
            _abi.check(_abi.lib.cpl_lagrangian_grad(B * 2 * nf, n, m, nnz, _ptr(csc[0]), _ptr(csc[1]), _ptr(csc[2]),
                                                    _ptr(o["grad"]), _ptr(o["jac"]), _ptr(yc), 2 * nf, _ptr(gL),
                                                    stream()))
        return gL, h

    def kkt_device(M, A, r1, r2, mu, dwl, active):
        """cpl_kkt_solve: factorise + solve on the device; returns (dw, dy, delta_w, solve_primal)."""
        Mc, Ac, r1c = M.contiguous(), A.contiguous(), r1.contiguous()
        act_u8 = active.to(torch.uint8)
        dw = torch.empty(B, nw, dtype=dt, device=dev)
        dy = torch.empty(B, m, dtype=dt, device=dev)
        delta_w = torch.empty(B, dtype=dt, device=dev)
        delta_c = torch.empty(B, dtype=dt, device=dev)
        info = torch.empty(B, dtype=torch.int32, device=dev)
        _abi.check(_abi.lib.cpl_kkt_solve(0, B, nw, m, _ptr(Mc), _ptr(Ac), _ptr(r1c), _ptr(r2.contiguous()),
                                          _ptr(mu.contiguous()), _ptr(dwl.contiguous()), _ptr(act_u8), _ptr(dw),
                                          _ptr(dy), _ptr(delta_w), _ptr(delta_c), _ptr(info), _ptr(kkt_ws),
                                          stream()))

        def solve_primal(r2v, mask=None):
            """Second-order correction: the kept factors, another r2; only the instances in mask
            (default: the factorised ones) are solved, the others get 0 and cost nothing."""
            out_dw = torch.empty(B, nw, dtype=dt, device=dev)
            out_dy = torch.empty(B, m, dtype=dt, device=dev)
            msk = act_u8 if mask is None else mask.to(torch.uint8)
            _abi.check(_abi.lib.cpl_kkt_solve(1, B, nw, m, _ptr(Mc), _ptr(Ac), _ptr(r1c), _ptr(r2v.contiguous()),
                                              None, None, _ptr(msk), _ptr(out_dw), _ptr(out_dy), None, None, None,
                                              _ptr(kkt_ws), stream()))
            return out_dw

        return dw, dy, delta_w, solve_primal

    def kkt_host(M, A, r1, r2, mu, dwl, active):
        """The same step as cpl_kkt_solve from torch's dense factorisations (host tensors), step for
        step: QR of A^T = [Y Z] [R; 0], delta_c on R's diagonal where |R_jj| < 1e-10 |R|max, the
        reduced Hessian Z^T M Z with the inertia test = its Cholesky (pivots at or below
        _PIVOT_REL |M|max count as zero eigenvalues), dw = Y R^-T q2 + Z p_z, R dy = Y^T (q1 - M dw),
        one refinement step when A has full rank."""
        Qf, Rf = torch.linalg.qr(A.transpose(1, 2), mode="complete")
        Y, Z = Qf[:, :, :m], Qf[:, :, m:]
        R = Rf[:, :m, :m].clone()
        Rd = R.diagonal(dim1=1, dim2=2)
        rmax = Rd.abs().amax(1) if m else zeros_B
        dc = 1e-8 * mu ** 0.25 * torch.where(rmax > 0, rmax, torch.ones_like(rmax))
        small = ~(Rd.abs() >= 1e-10 * rmax[:, None]) | (rmax[:, None] == 0)
        rank_def = small.any(1) if m else torch.zeros(B, dtype=torch.bool)
        delta_c = torch.where(rank_def, dc, zeros_B)
        Rd.copy_(torch.where(small, Rd + torch.where(Rd < 0, -dc[:, None], dc[:, None]), Rd))
        Hr = Z.transpose(1, 2) @ M @ Z
        Hr = 0.5 * (Hr + Hr.transpose(1, 2))
        nz = nw - m
        eye_z = torch.eye(nz, dtype=dt)
        piv_tol = _PIVOT_REL * M.diagonal(dim1=1, dim2=2).abs().amax(1)

        def chol(dw_):
            Lf, inf_ = torch.linalg.cholesky_ex(Hr + dw_[:, None, None] * eye_z)
            if nz:
                inf_ = torch.where((inf_ == 0) & ((Lf.diagonal(dim1=1, dim2=2) ** 2).amin(1) <= piv_tol),
                                   torch.ones_like(inf_), inf_)
            return Lf, inf_

        delta_w = zeros_B.clone()
        L1, info1 = chol(delta_w)
        for _ in range(64):
            bad = info1 != 0
            if not bool(bad.any()):
                break
            first_dw = torch.where(dwl == 0, torch.full_like(delta_w, 1e-4), torch.clamp(dwl / 3.0, min=1e-20))
            grow = delta_w * torch.where(dwl == 0, 100.0, 8.0)
            delta_w = torch.where(bad, torch.where(delta_w == 0, first_dw, grow), delta_w)
            L1n, info1n = chol(delta_w)
            L1 = torch.where(bad[:, None, None], L1n, L1)
            info1 = torch.where(bad, info1n, info1)
        Mw = M + delta_w[:, None, None] * eye_w

        def solve(q1, q2):
            py = torch.linalg.solve_triangular(R.transpose(1, 2), q2.unsqueeze(2), upper=False)
            dw_ = Y @ py
            if nz:
                pz = torch.cholesky_solve(Z.transpose(1, 2) @ (q1.unsqueeze(2) - Mw @ dw_), L1)
                dw_ = dw_ + Z @ pz
            dy_ = torch.linalg.solve_triangular(R, Y.transpose(1, 2) @ (q1.unsqueeze(2) - Mw @ dw_), upper=True)
            return dw_.squeeze(2), dy_.squeeze(2)

        def refined(q1, q2):
            d1, d2 = solve(q1, q2)
            e1 = q1 - (Mw @ d1.unsqueeze(2)).squeeze(2) - (A.transpose(1, 2) @ d2.unsqueeze(2)).squeeze(2)
            e2 = q2 - (A @ d1.unsqueeze(2)).squeeze(2)
            c1, c2 = solve(e1, e2)
            keep = rank_def[:, None]
            return torch.where(keep, d1, d1 + c1), torch.where(keep, d2, d2 + c2)

        dw, dy = refined(r1, r2)
        return dw, dy, delta_w, lambda r2v, mask=None: refined(r1, r2v)[0]

    kkt = kkt_device if use_hip else kkt_host


    def errors(o, wv, yv, zl, zu):
        A_ = jac_w(o["J"])
        gw = torch.cat([o["grad"][:, free], zeros_I], 1)
        c_ = cons(o["g"], wv[:, nf:])
        dual = gw + (A_.transpose(1, 2) @ yv.unsqueeze(2)).squeeze(2) - zl + zu
        cl = torch.where(hasL, (wv - wl0) * zl, torch.zeros_like(wv))
        cu = torch.where(hasU, (wu0 - wv) * zu, torch.zeros_like(wv))
        s_max = 100.0
        zsum = zl.abs().sum(1) + zu.abs().sum(1)
        sd = torch.clamp((yv.abs().sum(1) + zsum) / max(m + nbounds, 1), min=s_max) / s_max
        sc = torch.clamp(zsum / max(nbounds, 1), min=s_max) / s_max
        d_inf = dual.abs().amax(1)
        c_inf = c_.abs().amax(1) if m else zeros_B
        base = torch.maximum(d_inf / sd, c_inf)
        return {"A": A_, "gw": gw, "c": c_, "d_inf": d_inf, "base": base, "cl": cl, "cu": cu, "sc": sc,
                "err0": torch.maximum(base, torch.maximum(cl.amax(1), cu.amax(1)) / sc)}

    def err_mu(E, muv):
        comp_mu = torch.maximum((E["cl"] - torch.where(hasL, muv[:, None], 0.0)).abs().amax(1),
                                (E["cu"] - torch.where(hasU, muv[:, None], 0.0)).abs().amax(1))
        return torch.maximum(E["base"], comp_mu / E["sc"])

    def reset_filter(mask, ft, fp, fc):
        return (torch.where(mask[:, None], torch.full_like(ft, float("inf")), ft),
                torch.where(mask[:, None], torch.full_like(fp, float("inf")), fp),
                torch.where(mask, torch.zeros_like(fc), fc))

    def max_step(v, dv, lo_mask, lo, tau):
        r = torch.where(lo_mask & (dv < 0), -tau[:, None] * (v - lo) / torch.where(dv < 0, dv, -1.0),
                        torch.full_like(v, float("inf")))
        return torch.clamp(r.amin(1), max=1.0)

    # ---- starting point: x pushed into its bounds, slacks = g_I(x) pushed into theirs
    Xs = unpack(push(torch.cat([Xbase[:, free], zeros_I], 1)))
    cur0 = evaluate(Xs)
    w0 = push(torch.cat([Xs[:, free], cur0["g"][:, I]], 1))
    zL0 = torch.where(hasL, torch.ones_like(w0), torch.zeros_like(w0))
    zU0 = torch.where(hasU, torch.ones_like(w0), torch.zeros_like(w0))
    theta0 = cons(cur0["g"], w0[:, nf:]).abs().sum(1)
    theta_max = 1e4 * theta0.clamp(min=1.0)
    theta_min = 1e-4 * theta0.clamp(min=1.0)
    # least-squares constraint multipliers (IPOPT constr_mult_init_max = 1e3)
    A0 = jac_w(cur0["J"])
    gw0 = torch.cat([cur0["grad"][:, free], zeros_I], 1)
    L0, info0 = torch.linalg.cholesky_ex(A0 @ A0.transpose(1, 2) + 1e-12 * eye_m)
    y0 = -torch.cholesky_solve(A0 @ (gw0 - zL0 + zU0).unsqueeze(2), L0).squeeze(2)
    y0 = torch.where(((y0.abs().amax(1) <= 1e3) & (info0 == 0)).unsqueeze(1), y0, torch.zeros_like(y0))

    # persistent state: the (captured) iteration reads these and writes them back in place
    S = {
        "w": w0.contiguous(), "y": y0.contiguous(), "zL": zL0, "zU": zU0,
        "mu": torch.full((B,), mu_init, dtype=dt, device=dev),
        "active": torch.ones(B, dtype=torch.bool, device=dev),
        "status": torch.full((B,), STATUS_MAX_ITER, dtype=torch.int64, device=dev),
        "iters": torch.zeros(B, dtype=torch.int64, device=dev),
        "acc": torch.zeros(B, dtype=torch.int64, device=dev),
        "filt_t": torch.full((B, FMAX), float("inf"), dtype=dt, device=dev),
        "filt_p": torch.full((B, FMAX), float("inf"), dtype=dt, device=dev),
        "fcount": torch.zeros(B, dtype=torch.int64, device=dev),
        "dwl": zeros_B.clone(),
        "f": cur0["f"].clone(), "grad": cur0["grad"].clone(), "g": cur0["g"].clone(), "J": cur0["J"].clone(),
        "d_inf": zeros_B.clone(),
        "Hq": eye_f.repeat(B, 1, 1) if use_bfgs else None,
        "hq_init": torch.zeros(B, dtype=torch.bool, device=dev),
    }

    def check(E):
        """Convergence test at the current iterate; updates status / active / acc; returns active."""
        active = S["active"]
        e0 = E["err0"]
        done_now = active & (e0 <= tol)
        acc = torch.where(active & (e0 <= acceptable_tol), S["acc"] + 1, torch.zeros_like(S["acc"]))
        acc_now = active & ~done_now & (acc >= acceptable_iter)
        status = torch.where(done_now, torch.full_like(S["status"], STATUS_OPTIMAL),
                             torch.where(acc_now, torch.full_like(S["status"], STATUS_ACCEPTABLE), S["status"]))
        active = active & ~done_now & ~acc_now
        S["acc"].copy_(acc)
        S["status"].copy_(status)
        S["active"].copy_(active)
        S["d_inf"].copy_(E["d_inf"])
        return active

    def step():
        """One lock-step iteration of every instance; no host synchronisation (graph-capturable)."""
        w, y, zL, zU, mu = S["w"], S["y"], S["zL"], S["zU"], S["mu"]
        cur = {"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}
        if use_hip:  # optimality error, convergence test and barrier update: one fused launch
            A = jac_w(cur["J"], S["active"])
            gradw = torch.cat([cur["grad"][:, free], zeros_I], 1)
            c = cons(cur["g"], w[:, nf:])
            E = {k: torch.empty(B, dtype=dt, device=dev) for k in ("d_inf", "err0", "base")}
            mu_o = torch.empty(B, dtype=dt, device=dev)
            ft, fp = torch.empty_like(S["filt_t"]), torch.empty_like(S["filt_p"])
            fc = torch.empty_like(S["fcount"])
            _abi.check(_abi.lib.cpl_ipm_optimality(
                B, nw, m, FMAX, nbounds, tol, acceptable_tol, acceptable_iter, _ptr(A), _ptr(gradw), _ptr(c), _ptr(w),
                _ptr(y), _ptr(zL), _ptr(zU), _ptr(hasL_u8), _ptr(hasU_u8), _ptr(wl0), _ptr(wu0), _ptr(mu),
                _ptr(S["filt_t"]), _ptr(S["filt_p"]), _ptr(S["fcount"]), _ptr(S["active"]), _ptr(S["status"]),
                _ptr(S["acc"]), _ptr(E["d_inf"]), _ptr(E["err0"]), _ptr(E["base"]), _ptr(mu_o), _ptr(ft), _ptr(fp),
                _ptr(fc), stream()))
            S["d_inf"].copy_(E["d_inf"])
            active = S["active"].clone()
            mu = mu_o
        else:
            E = errors(cur, w, y, zL, zU)
            active = check(E).clone()
            A, gradw, c = E["A"], E["gw"], E["c"]
            # ---- monotone barrier update (two rounds per iteration), filter reset where mu changed
            ft, fp, fc = S["filt_t"], S["filt_p"], S["fcount"]
            for _ in range(2):
                upd = active & (err_mu(E, mu) <= 10.0 * mu) & (mu > tol / 10.0)
                mu = torch.where(upd, torch.clamp(torch.minimum(0.2 * mu, mu ** 1.5), min=tol / 10.0), mu)
                ft, fp, fc = reset_filter(upd, ft, fp, fc)
        tau = torch.clamp(1.0 - mu, min=0.99)

        def primal_step(d):  # fraction to the boundary along d from w
            if use_hip:
                out = torch.empty(B, dtype=dt, device=dev)
                _abi.check(_abi.lib.cpl_ipm_max_step(B, nw, _ptr(w), _ptr(d.contiguous()), None, None, _ptr(hasL_u8),
                                                     _ptr(hasU_u8), _ptr(wl0), _ptr(wu0), _ptr(tau), _ptr(out),
                                                     stream()))
                return out
            return torch.minimum(max_step(w, d, hasL, wl0, tau), max_step(-w, -d, hasU, -wu0, tau))

        gLfd = hfd = None
        if use_bfgs:
            Hblk = S["Hq"]
        elif analytic_H:  # the exact Hessian of the Lagrangian, one thread per entry
            Hblk = torch.empty(B, nf, nf, dtype=dt, device=dev)
            _abi.check(_abi.lib.cpl_lagrangian_hessian(ctypes.byref(problem.desc()), B, _ptr(unpack(w)),
                                                       _ptr(y.contiguous()), _ptr(S["active"]), _ptr(free_i32), nf,
                                                       _ptr(Hblk), stream()))
        elif use_hip:  # raw central differences here, symmetrised inside the Newton setup kernel
            gLfd, hfd = fd_grads_dev(unpack(w), y)
            Hblk = torch.empty(B, nf, nf, dtype=dt, device=dev)
            _abi.check(_abi.lib.cpl_ipm_fd_hessian_raw(B, n, nf, _ptr(free), _ptr(gLfd), _ptr(hfd), _ptr(Hblk),
                                                       _ptr(S["active"]), stream()))
        else:
            # host path: the evaluator's own analytic Hessian when it has one (the oracle's restatement
            # of cpl_lagrangian_hessian, so the CPU solve takes the device's exact-Hessian steps)
            Hblk = ev.hessian(unpack(w), y, free) if (hessian == "exact" and hasattr(ev, "hessian")) else None
            if Hblk is None:
                Hblk = fd_hessian(unpack(w), y)
        if use_hip:  # Newton system: one fused launch (csrc/cpl_ipm.hip)
            M = torch.empty(B, nw, nw, dtype=dt, device=dev)
            r1, gphi, mr_diag = (torch.empty(B, nw, dtype=dt, device=dev) for _ in range(3))
            r2 = torch.empty(B, m, dtype=dt, device=dev)
            theta_k, phi_k = torch.empty(B, dtype=dt, device=dev), torch.empty(B, dtype=dt, device=dev)
            _abi.check(_abi.lib.cpl_ipm_newton_setup(
                B, nw, m, nf, _ptr(w), _ptr(zL), _ptr(zU), _ptr(gradw), _ptr(A), _ptr(y), _ptr(c),
                _ptr(cur["f"]), _ptr(mu), _ptr(hasL_u8), _ptr(hasU_u8), _ptr(wl0), _ptr(wu0),
                None if Hblk is None else _ptr(Hblk.contiguous()), 0 if (use_bfgs or analytic_H) else 1,
                _ptr(M), _ptr(r1), _ptr(r2), _ptr(gphi), _ptr(mr_diag), _ptr(theta_k), _ptr(phi_k),
                _ptr(S["active"]) if not use_bfgs else None, stream()))
        else:
            dl = torch.where(hasL, w - wl0, torch.ones_like(w))
            du = torch.where(hasU, wu0 - w, torch.ones_like(w))
            Sig = torch.where(hasL, zL / dl, torch.zeros_like(w)) + torch.where(hasU, zU / du, torch.zeros_like(w))
            gphi = gradw - torch.where(hasL, mu[:, None] / dl, torch.zeros_like(w)) + \
                torch.where(hasU, mu[:, None] / du, torch.zeros_like(w))
            r1 = -(gphi + (A.transpose(1, 2) @ y.unsqueeze(2)).squeeze(2))
            r2 = -c
            M = torch.diag_embed(Sig)
            M[:, :nf, :nf] += Hblk
            mr_diag = Sig + mu.sqrt()[:, None] * torch.clamp(w.abs(), min=1.0) ** -2
            theta_k = c.abs().sum(1)
            phi_k = cur["f"] + barrier(w, mu)
        dw, dy, delta_w, solve_primal = kkt(M, A, r1, r2, mu, S["dwl"], active)
        if use_hip:  # multiplier steps, fraction-to-boundary steps, gd, switching flag: one launch
            dzL, dzU = torch.empty_like(w), torch.empty_like(w)
            a_max, a_z, gd = (torch.empty(B, dtype=dt, device=dev) for _ in range(3))
            switch_ok = torch.empty(B, dtype=torch.bool, device=dev)
            _abi.check(_abi.lib.cpl_ipm_post_step(
                B, nw, _ptr(w), _ptr(dw.contiguous()), _ptr(zL), _ptr(zU), _ptr(gphi), _ptr(mu), _ptr(tau),
                _ptr(hasL_u8), _ptr(hasU_u8), _ptr(wl0), _ptr(wu0), _ptr(theta_k), _ptr(theta_min), _ptr(active),
                _ptr(delta_w.contiguous()), _ptr(S["dwl"]), _ptr(dzL), _ptr(dzU), _ptr(a_max), _ptr(a_z), _ptr(gd),
                _ptr(switch_ok), stream()))
            dwl = S["dwl"]
        else:
            dwl = torch.where(active, delta_w, S["dwl"])
            dzL = torch.where(hasL, mu[:, None] / dl - zL - zL / dl * dw, torch.zeros_like(w))
            dzU = torch.where(hasU, mu[:, None] / du - zU + zU / du * dw, torch.zeros_like(w))
            a_max = primal_step(dw)
            a_z = torch.minimum(max_step(zL, dzL, hasL, 0.0, tau), max_step(zU, dzU, hasU, 0.0, tau))
            gd = (gphi * dw).sum(1)
            switch_ok = (theta_k <= theta_min) & (gd < 0)

        # ---- filter line search (IPOPT: gamma_theta 1e-5, gamma_phi 1e-8, delta 1, s_theta 1.1,
        # s_phi 2.3, eta_phi 1e-8, theta_min/max = 1e-4/1e4 max(1, theta_0)), second-order
        # corrections on the first trial; fixed trip counts, masked acceptance
        # line-search state (fresh tensors: the device path updates them in place)
        st = {"searching": active.clone(), "f": cur["f"].clone(), "g": cur["g"].clone(), "w": w.clone(),
              "alpha": zeros_B.clone(), "aug": torch.zeros(B, dtype=torch.bool, device=dev)}

        def judge(wt, o, al):  # o: {"f", "g"} at the trial points
            th = cons(o["g"], wt[:, nf:]).abs().sum(1)
            ph = o["f"] + barrier(wt, mu)
            fin = torch.isfinite(ph) & torch.isfinite(th)
            in_filter = ((th[:, None] <= (1.0 - 1e-5) * ft) | (ph[:, None] <= fp - 1e-8 * ft)).all(1)
            ftype = switch_ok & (al * (-gd).clamp(min=0.0) ** 2.3 > theta_k ** 1.1)
            armijo = ph <= phi_k + 1e-8 * al * gd
            suff = (th <= (1.0 - 1e-5) * theta_k) | (ph <= phi_k - 1e-8 * theta_k)
            ok = fin & (th <= theta_max) & in_filter & torch.where(ftype, armijo, suff)
            return ok, ~(ftype & armijo), th

        def take(mask, wt, o, al, aug_mask):
            st["f"] = torch.where(mask, o["f"], st["f"])
            st["g"] = torch.where(mask[:, None], o["g"], st["g"])
            st["w"] = torch.where(mask[:, None], wt, st["w"])
            st["alpha"] = torch.where(mask, al, st["alpha"])
            st["aug"] = torch.where(mask, aug_mask, st["aug"])
            st["searching"] = st["searching"] & ~mask

        if use_hip:  # the fused kernels of csrc/cpl_ipm.hip (one launch per trial for each)
            sw_ok = switch_ok.contiguous()
            ftc, fpc = ft.contiguous(), fp.contiguous()

            def trial(d, al, mask):
                """w_t = w + al d; the evaluation point takes w_t where mask, else the state's w."""
                wt_ = torch.empty_like(w)
                Xt = torch.empty(B, n, dtype=dt, device=dev)
                _abi.check(_abi.lib.cpl_ipm_trial_point(B, n, nf, nw, _ptr(free), _ptr(fixed), _ptr(Xbase), _ptr(w),
                                                        _ptr(d.contiguous()), _ptr(al.contiguous()),
                                                        _ptr(mask.contiguous()), _ptr(st["w"]), _ptr(wt_), _ptr(Xt),
                                                        stream()))
                return wt_, evaluate_fg(Xt)

            def judge_take(wt_, o_, al, extra=None, mode=0):
                """IPOPT's acceptance test + take for searching (& extra) instances; (ok, theta).
                mode 1: the feasibility step's test; mode 2: take unconditionally."""
                th_ = torch.empty(B, dtype=dt, device=dev)
                ok_ = torch.empty(B, dtype=torch.bool, device=dev)
                _abi.check(_abi.lib.cpl_ipm_judge_take(
                    B, nw, m, nf, FMAX, _ptr(row_slack), _ptr(gl), _ptr(hasL_u8), _ptr(hasU_u8), _ptr(wl0), _ptr(wu0),
                    _ptr(wt_), _ptr(o_["f"].contiguous()), _ptr(o_["g"].contiguous()), _ptr(al.contiguous()),
                    _ptr(mu.contiguous()), _ptr(theta_k.contiguous()), _ptr(phi_k.contiguous()), _ptr(gd.contiguous()),
                    _ptr(sw_ok), _ptr(theta_max), _ptr(ftc), _ptr(fpc), None if extra is None else _ptr(extra.contiguous()),
                    _ptr(st["searching"]), _ptr(st["f"]), _ptr(st["g"]), _ptr(st["w"]), _ptr(st["alpha"]),
                    _ptr(st["aug"]), _ptr(th_), _ptr(ok_), mode, stream()))
                return ok_, th_
        else:
            def trial(d, al, mask):
                wt_ = w + al[:, None] * d
                return wt_, evaluate_fg(unpack(torch.where(mask[:, None], wt_, st["w"])))

            def judge_take(wt_, o_, al, extra=None):
                ok_, augm_, th_ = judge(wt_, o_, al)
                take(st["searching"] & ok_ & (True if extra is None else extra), wt_, o_, al, augm_)
                return ok_, th_

        alpha = a_max
        wt, o = w, cur
        for ls in range(max(1, max_ls)):
            wt, o = trial(dw, alpha, st["searching"])
            ok, th = judge_take(wt, o, alpha)
            if ls == 0 and max_soc > 0:
                soc = st["searching"] & (th >= theta_k)
                c_soc, a_soc, th_old = c, alpha, theta_k
                ct = cons(o["g"], wt[:, nf:])
                for _ in range(max_soc):
                    c_soc = a_soc[:, None] * c_soc + ct
                    dws = solve_primal(-c_soc, soc)  # only the instances that try a correction
                    a_soc = primal_step(dws)
                    ws, os_ = trial(dws, a_soc, soc)
                    oks, ths = judge_take(ws, os_, alpha, soc)
                    soc = soc & ~oks & (ths <= 0.99 * th_old)  # kappa_soc = 0.99
                    th_old = ths
                    ct = cons(os_["g"], ws[:, nf:])
            alpha = torch.where(st["searching"], 0.5 * alpha, alpha)
        # no acceptable trial: a feasibility step stands in for IPOPT's restoration phase —
        # min 1/2 dw^T (Sigma + sqrt(mu) D_R^2) dw s.t. A dw = -c (D_R = diag(1 / max(1, |w|)),
        # IPOPT's restoration proximity weight), fraction to the boundary, taken when it cuts the
        # violation by 10 %; the multipliers stay.  Otherwise the last trial.  Either way the
        # instance's filter restarts.  (The KKT kernel skips the instances outside the mask.)
        failed = st["searching"].clone()
        if use_hip:  # persistent zero matrix: only its diagonal changes (no 8 192 x nw x nw fill)
            Mr_buf.diagonal(dim1=1, dim2=2).copy_(mr_diag)
            Mr = Mr_buf
        else:
            Mr = torch.diag_embed(mr_diag)
        dwr = kkt(Mr, A, torch.zeros_like(w), -c, mu, zeros_B, failed)[0]
        ar = primal_step(dwr)
        wr, orr = trial(dwr, ar, failed)
        if use_hip:
            ok_r, _ = judge_take(wr, orr, zeros_B, failed, mode=1)
            rest = failed & ok_r
            judge_take(wt, o, 2.0 * alpha, None, mode=2)
        else:
            thr = cons(orr["g"], wr[:, nf:]).abs().sum(1)
            rest = failed & torch.isfinite(thr) & torch.isfinite(orr["f"]) & (thr <= 0.9 * theta_k)
            take(rest, wr, orr, zeros_B, torch.zeros_like(failed))
            take(st["searching"], wt, o, 2.0 * alpha, torch.zeros_like(failed))
        w_new = st["w"]
        al = st["alpha"]
        # the accepted points with their derivatives: one full evaluation (trials carried f and g only)
        new = evaluate(unpack(w_new))
        if use_hip and not use_bfgs:  # accept + state write-back: one launch, plus masked row copies
            _abi.check(_abi.lib.cpl_ipm_accept(
                B, nw, m, FMAX, _ptr(active), _ptr(st["aug"]), _ptr(failed), _ptr(rest), _ptr(al), _ptr(a_z),
                _ptr(theta_k), _ptr(phi_k), _ptr(ft), _ptr(fp), _ptr(fc), _ptr(w_new), _ptr(dy.contiguous()),
                _ptr(dzL), _ptr(dzU), _ptr(mu), _ptr(hasL_u8), _ptr(hasU_u8), _ptr(wl0), _ptr(wu0), _ptr(S["w"]),
                _ptr(S["y"]), _ptr(S["zL"]), _ptr(S["zU"]), _ptr(S["mu"]), _ptr(S["iters"]), _ptr(S["filt_t"]),
                _ptr(S["filt_p"]), _ptr(S["fcount"]), stream()))
            for k in ("f", "grad", "g", "J"):
                _abi.check(_abi.lib.cpl_ipm_masked_rows(B, S[k].numel() // B, _ptr(active), _ptr(new[k].contiguous()),
                                                        _ptr(S[k]), stream()))
            if verbose > 1:
                verbose_line(E, mu, a_max, al, dw, dy, delta_w, cur)
            return
        a_z = torch.where(rest, zeros_B, a_z)
        addm = st["aug"] & active
        fi = fslot == torch.remainder(fc, FMAX)[:, None]
        ft = torch.where(addm[:, None] & fi, ((1.0 - 1e-5) * theta_k)[:, None], ft)
        fp = torch.where(addm[:, None] & fi, (phi_k - 1e-8 * theta_k)[:, None], fp)
        fc = fc + addm.to(fc.dtype)
        ft, fp, fc = reset_filter(failed, ft, fp, fc)

        # ---- accept: primal, multipliers, bound multipliers (kappa_Sigma safeguard)
        act = active[:, None]
        y_new = torch.where(act, y + al[:, None] * dy, y)
        zL_new = torch.where(act & hasL, zL + a_z[:, None] * dzL, zL)
        zU_new = torch.where(act & hasU, zU + a_z[:, None] * dzU, zU)
        dln = torch.where(hasL, w_new - wl0, torch.ones_like(w))
        dun = torch.where(hasU, wu0 - w_new, torch.ones_like(w))
        zL_new = torch.where(act & hasL, torch.minimum(torch.maximum(zL_new, mu[:, None] / (1e10 * dln)),
                                                       1e10 * mu[:, None] / dln), zL_new)
        zU_new = torch.where(act & hasU, torch.minimum(torch.maximum(zU_new, mu[:, None] / (1e10 * dun)),
                                                       1e10 * mu[:, None] / dun), zU_new)

        if use_bfgs:  # damped BFGS update over x_free (both Lagrangian gradients at the new y)
            Hq = S["Hq"]
            sk = (w_new - w)[:, :nf]
            JTy_new = (new["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
            JTy_old = (cur["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
            yk = (new["grad"] + JTy_new)[:, free] - (cur["grad"] + JTy_old)[:, free]
            sy = (sk * yk).sum(1)
            ss = (sk * sk).sum(1)
            first = active & ~S["hq_init"] & (sy > 0) & (ss > 0)
            sigma0 = torch.where(first, sy / torch.where(ss > 0, ss, 1.0), torch.ones_like(sy))
            Hq = torch.where(first[:, None, None], sigma0[:, None, None] * eye_f, Hq)
            S["hq_init"].copy_(S["hq_init"] | first)
            Hs = (Hq @ sk.unsqueeze(2)).squeeze(2)
            sHs = (sk * Hs).sum(1)
            theta = torch.where(sy >= 0.2 * sHs, torch.ones_like(sy),
                                0.8 * sHs / torch.where(sHs - sy != 0, sHs - sy, 1.0))
            r = theta[:, None] * yk + (1.0 - theta[:, None]) * Hs
            sr = (sk * r).sum(1)
            upd = active & (ss > 1e-30) & (sHs > 0) & (sr > 0)
            Hn = Hq - Hs.unsqueeze(2) * Hs.unsqueeze(1) / torch.where(upd, sHs, 1.0)[:, None, None] + \
                r.unsqueeze(2) * r.unsqueeze(1) / torch.where(upd, sr, 1.0)[:, None, None]
            S["Hq"].copy_(torch.where(upd[:, None, None], 0.5 * (Hn + Hn.transpose(1, 2)), Hq))

        # ---- write the state back in place
        S["w"].copy_(torch.where(act, w_new, w))
        S["y"].copy_(y_new)
        S["zL"].copy_(zL_new)
        S["zU"].copy_(zU_new)
        S["mu"].copy_(mu)
        S["iters"].copy_(S["iters"] + active.to(torch.int64))
        S["filt_t"].copy_(ft)
        S["filt_p"].copy_(fp)
        S["fcount"].copy_(fc)
        S["dwl"].copy_(dwl)
        for k in ("f", "grad", "g", "J"):
            S[k].copy_(torch.where(active.view(-1, *([1] * (S[k].dim() - 1))), new[k], S[k]))
        if verbose > 1:
            verbose_line(E, mu, a_max, al, dw, dy, delta_w, cur)

    def verbose_line(E, mu, a_max, al, dw, dy, delta_w, cur):
        b = int(verbose) - 2
        print(f"   [{b}] mu={float(mu[b]):.2e} err0={float(E['err0'][b]):.2e} a_max={float(a_max[b]):.2e} "
              f"alpha={float(al[b]):.2e} dw={float(dw[b].abs().max()):.2e} dy={float(dy[b].abs().max()):.2e} "
              f"dW={float(delta_w[b]):.1e} f={float(cur['f'][b]):.6e} d_inf={float(E['d_inf'][b]):.2e} "
              f"c_inf={float(E['base'][b]):.2e} argdw={int(dw[b].abs().argmax())}")

    # ---- drive the iterations
    it_run = 0
    replay = step
    per_step_evals = 0
    if use_graph and max_iter > 0:
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up iteration (executed): per-stream state, allocator pools
            step()
        torch.cuda.current_stream(dev).wait_stream(side)
        it_run = 1
        e0 = n_eval
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            step()
        per_step_evals = n_eval - e0
        n_eval = e0
        replay = gr.replay
    if use_hip:
        # termination test without stalling the device: after every iteration "any active" goes to
        # a pinned host slot behind an event; the host reads the previous iteration's slot (normally
        # landed already) while the current iteration runs — at most one iteration past the end
        # (a no-op: every update is masked by the active flags)
        flag = torch.zeros(2, dtype=torch.bool).pin_memory()
        evs = [torch.cuda.Event(), torch.cuda.Event()]
        if not bool(S["active"].any()):
            max_iter = it_run
        start = it_run
        while it_run < max_iter:
            replay()
            n_eval += per_step_evals
            it_run += 1
            k = it_run & 1
            flag[k].copy_(S["active"].any(), non_blocking=True)
            evs[k].record()
            if verbose:
                print(f"it {it_run:4d} active {int(S['active'].sum())}")
            if it_run - start >= 2:  # the previous iteration of this loop recorded its flag
                evs[k ^ 1].synchronize()
                if not bool(flag[k ^ 1]):
                    break
    else:
        while it_run < max_iter:
            if it_run % max(1, check_every) == 0 and not bool(S["active"].any()):
                break
            replay()
            n_eval += per_step_evals
            it_run += 1
            if verbose:
                print(f"it {it_run:4d} active {int(S['active'].sum())}")
    # final convergence test at the last iterate
    check(errors({"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}, S["w"], S["y"], S["zL"], S["zU"]))
    # IPOPT honor_original_bounds: the final point is projected back into the unrelaxed bounds and
    # its objective / constraint values reported there
    Xf = torch.minimum(torch.maximum(unpack(S["w"]), xl), xu).contiguous()
    fin = evaluate_fg(Xf)
    g = fin["g"]
    viol = torch.clamp(torch.maximum(gl - g, g - gu), min=0.0).amax(1) if m else zeros_B
    return BatchSolveResult(x=Xf, y=S["y"], status=S["status"], iterations=S["iters"],
                            objective=fin["f"].clone(), primal_inf=viol, dual_inf=S["d_inf"], evaluations=n_eval,
                            iterations_run=it_run, graph=use_graph)
