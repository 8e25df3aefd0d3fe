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
    (cpl_lagrangian_grad); or (hessian="limited-memory", what IFOPT configures) IPOPT's limited-memory BFGS
    model initialised like IPOPT's scalar1 = s'y / s's;
  * Newton step (cpl_kkt_solve, csrc/cpl_kkt.hip): null-space method on a Householder QR of A^T
    (A = [J_free | -P]) with IPOPT's inertia correction on the device — the KKT matrix has inertia
    (nw+, m-, 0) iff A has full row rank and the reduced Hessian Z^T (W + Sigma) Z is positive
    definite, so its Cholesky is the inertia test (failure -> delta_w with IPOPT's schedule); a
    rank-deficient A (the single-contact torque about the force line) gets delta_c; one step of
    iterative refinement.  Host tensors (the solver's logic under test on the CPU) take the same
    step from torch's dense factorisations (projector form of the null-space method);
  * fraction-to-the-boundary rule (tau = max(0.99, 1 - mu)), monotone Fiacco-McCormick barrier
    update (kappa_mu = 0.2, theta_mu = 1.5, kappa_eps = 10, up to 6 decreases per iteration, floor
    min(tol, 1e-4) / 11) with a filter reset, IPOPT's filter line search (switching condition, Armijo
    on the barrier objective for f-type steps, filter augmentation after h-type steps, Compare_le
    round-off tolerance, obj_max_inc) backtracking while alpha > alpha_min with up to max_soc
    second-order corrections on the first trial, tiny steps, the soft restoration step, and IPOPT's
    restoration phase (MinC_1Nrm: min rho |p + n|_1 + eta/2 |D_R (x - x_R)|^2 s.t. c(w) - p + n = 0
    with its own barrier parameter, filter and line search) where the search fails — unless the
    point is already acceptable, where the solve stops (STOP_AT_ACCEPTABLE_POINT);
    kappa_Sigma = 1e10 safeguard on the bound multipliers;
  * termination on IPOPT's scaled optimality error (s_max = 100) <= tol, or <= acceptable_tol
    (1e-6) for 15 consecutive iterations.

Every evaluation — the iterate, each line-search trial point, the finite-difference points — is ONE
batched call of the evaluator for all instances (the device engine runs the trials after the first
inside one kernel, per instance).  Instances that converged stay in the batch (frozen), so every
launch keeps its shape.

Two implementations of the same iteration:
  * device tensors -> the native engine (csrc/cpl_solver.hip, C-ABI cpl_solver_*, NativeSolver
    below): the product callbacks (cpl_eval_batch with values-only Jacobian records), the Newton
    step in cpl_kkt_solve, the per-instance work in the cpl_ipm_* kernels and the glue in the
    engine's own kernels; the phases of the iteration captured once as HIP graphs and replayed, the
    host reading a few flag bytes per iteration.  No framework ops on the path;
  * host tensors -> this module's torch restatement over any evaluator's callbacks (the tests drive
    it with the oracle's): the checker of the device path — the same algorithm, step for step.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import _abi
from ._abi import INF

EPS = float(np.finfo(np.float64).eps)
LM_HIST, LM_MAX_SKIP = 6, 2  # IPOPT limited_memory_max_history / limited_memory_max_skipping

BIG = INF / 10.0  # |bound| >= 1e19 is infinite (IPOPT nlp_lower/upper_bound_inf)

STATUS_OPTIMAL = 0
STATUS_ACCEPTABLE = 1
STATUS_MAX_ITER = 2
STATUS_INFEASIBLE = 3     # the restoration phase converged: a point of local infeasibility
STATUS_RESTO_FAILED = 4   # the restoration phase converged twice to a feasible point the filter rejects, or
                          # it was called at an almost feasible point without a backup acceptable point
STATUS_NAMES = {STATUS_OPTIMAL: "optimal", STATUS_ACCEPTABLE: "acceptable", STATUS_MAX_ITER: "max_iter",
                STATUS_INFEASIBLE: "local_infeasibility", STATUS_RESTO_FAILED: "restoration_failed"}

# IPOPT's defaults (Waechter & Biegler 2006; IpFilterLSAcceptor / IpBacktrackingLineSearch /
# IpMonotoneMuUpdate / IpRestoMinC_1Nrm option defaults) that the iteration restates
GAMMA_TH, GAMMA_PHI, DELTA_SW, S_TH, S_PHI, ETA_PHI = 1e-5, 1e-8, 1.0, 1.1, 2.3, 1e-8  # filter / switching / Armijo
ALPHA_MIN_FRAC = 0.05      # alpha_min_frac
KAPPA_SOC = 0.99           # kappa_soc
OBJ_MAX_INC = 5.0          # obj_max_inc
KAPPA_SIGMA = 1e10         # kappa_sigma
BARRIER_TOL_FACTOR = 10.0  # barrier_tol_factor (kappa_epsilon)
COMPL_INF_TOL = 1e-4       # compl_inf_tol (the barrier parameter's floor: min(tol, compl_inf_tol) / 11)
MU_ROUNDS = 6              # barrier decreases per iteration (mu_allow_fast_monotone_decrease; 0.1 -> floor in 6)
TINY_STEP_TOL, TINY_STEP_Y_TOL = 10.0 * EPS, 1e-2  # tiny_step_tol, tiny_step_y_tol
RHO_R = 1000.0             # resto_penalty_parameter
KAPPA_RESTO = 0.9          # required_infeasibility_reduction
BOUND_MULT_RESET = 1000.0  # bound_mult_reset_threshold
SOFT_RESTO_FACTOR = 0.9999  # soft_resto_pderror_reduction_factor
MAX_SOFT_RESTO = 10         # max_soft_resto_iters
ALMOST_FEASIBLE = 1e-2      # BacktrackingLineSearch: no restoration phase at theta <= 1e-2 tol

FMAX = 64  # filter entries kept per instance (a ring)
SCALING_MAX_GRADIENT = 100.0  # nlp_scaling_max_gradient (nlp_scaling_method = gradient-based, IPOPT's default)
SCALING_MIN_VALUE = 1e-8      # nlp_scaling_min_value


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
    compactions: int = 0  # active-set compactions of the native engine (the batch shrank this often)
    final_rows: int = 0   # the native engine's lock-step batch size at the end (after compactions)
    restorations: object = None  # [B] int: restoration-phase entries per instance
    fallback: object = None  # [B] bool: x is the best feasible iterate, not the last (fallback_viol_tol)
    nan_jacobian: object = None  # [B] int: NaN Jacobian entries at the start point (taken as 0)

    @property
    def success(self):
        return self.status <= STATUS_ACCEPTABLE


_PIVOT_REL = 2.220446049250313e-16  # DBL_EPSILON: the KKT inertia test's zero-pivot level


class NativeSolver:
    """The native batched solve engine (csrc/cpl_solver.hip, C-ABI cpl_solver_*): the device path of
    batch_ipm_solve.  One handle per (problem template, batch, options): device buffers allocated
    once, the iteration captured once as a HIP graph and replayed on every solve."""

    def __init__(self, problem, batch, tol=1e-8, max_iter=3000, mu_init=0.1, acceptable_tol=1e-6,
                 acceptable_iter=15, max_ls=40, max_soc=4, hessian="exact", fd_step=1e-6, graph=True, compact=True,
                 ls_kernel=2, fallback_viol_tol=0.0, nlp_scaling="gradient-based", jacobian_regularization="pivot"):
        o = _abi.SolveOptions()
        _abi.lib.cpl_solve_options_default(ctypes.byref(o))
        o.max_iter, o.max_ls, o.max_soc, o.acceptable_iter = int(max_iter), int(max_ls), int(max_soc), int(acceptable_iter)
        o.tol, o.acceptable_tol, o.mu_init, o.fd_step = float(tol), float(acceptable_tol), float(mu_init), float(fd_step)
        o.hessian = {"exact": _abi.HESSIAN_EXACT, "limited-memory": _abi.HESSIAN_LIMITED_MEMORY,
                     "fd": _abi.HESSIAN_FD}[hessian]
        o.use_graph = 1 if graph else 0
        o.compact = 1 if compact else 0
        o.ls_kernel = int(ls_kernel)
        o.fallback_viol_tol = float(fallback_viol_tol)
        o.nlp_scaling = {"gradient-based": 1, "none": 0}[nlp_scaling]
        o.jacobian_regularization = {"pivot": 0, "ipopt": 1}[jacobian_regularization]
        self.problem, self.batch = problem, int(batch)
        self.desc = problem.desc()
        self.handle = ctypes.c_void_p()
        _abi.check(_abi.lib.cpl_solver_create(ctypes.byref(self.desc), self.batch, ctypes.byref(o),
                                              ctypes.byref(self.handle)))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _abi is not None and getattr(_abi, "lib", None) is not None:
            _abi.lib.cpl_solver_destroy(h)
            self.handle = None

    def solve(self, X0, mass=None, env_tag=None) -> "BatchSolveResult":
        import torch

        n, m, _ = self.problem.get_nlp_info()
        B, dev = self.batch, X0.device
        if X0.shape != (B, n) or X0.dtype != torch.float64 or not X0.is_cuda:
            raise ValueError(f"X0 must be a float64 CUDA tensor [{B}, {n}]")
        X0 = X0.contiguous()
        # the engine copies the masses / tags device-to-device: same device as X0, one per instance
        if mass is not None:
            if not torch.is_tensor(mass) or mass.device != dev or tuple(mass.shape) != (B,):
                raise ValueError(f"mass must be a tensor [{B}] on {dev}")
            mass = mass.to(torch.float64).contiguous()
        if env_tag is not None:
            if (not torch.is_tensor(env_tag) or env_tag.device != dev or tuple(env_tag.shape) != (B,)
                    or env_tag.dtype != torch.uint8):
                raise ValueError(f"env_tag must be a uint8 tensor [{B}] on {dev}")
            env_tag = env_tag.contiguous()
        x = torch.empty(B, n, dtype=torch.float64, device=dev)
        y = torch.empty(B, m, dtype=torch.float64, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        obj, pinf, dinf = (torch.empty(B, dtype=torch.float64, device=dev) for _ in range(3))
        it = ctypes.c_int32()
        ev = ctypes.c_int64()
        _abi.check(_abi.lib.cpl_solver_solve(
            self.handle, _ptr(X0), None if mass is None else _ptr(mass), None if env_tag is None else _ptr(env_tag),
            _ptr(x), _ptr(y), _ptr(status), _ptr(iters), _ptr(obj), _ptr(pinf), _ptr(dinf), ctypes.byref(it),
            ctypes.byref(ev), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        g = ctypes.c_int32()
        _abi.check(_abi.lib.cpl_solver_dims(self.handle, None, None, ctypes.byref(g)))
        nc, rows = ctypes.c_int32(), ctypes.c_int64()
        _abi.check(_abi.lib.cpl_solver_stats(self.handle, ctypes.byref(nc), ctypes.byref(rows)))
        self.compactions, self.final_rows = int(nc.value), int(rows.value)
        resto = torch.empty(B, dtype=torch.int64, device=dev)
        _abi.check(_abi.lib.cpl_solver_restorations(self.handle, _ptr(resto),
                                                    ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        fb = torch.empty(B, dtype=torch.uint8, device=dev)
        _abi.check(_abi.lib.cpl_solver_fallbacks(self.handle, _ptr(fb),
                                                 ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        nanj = torch.empty(B, dtype=torch.int32, device=dev)
        _abi.check(_abi.lib.cpl_solver_nan_jacobian(self.handle, _ptr(nanj),
                                                    ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        return BatchSolveResult(x=x, y=y, status=status.to(torch.int64), iterations=iters.to(torch.int64),
                                objective=obj, primal_inf=pinf, dual_inf=dinf, evaluations=int(ev.value),
                                iterations_run=int(it.value), graph=bool(g.value), compactions=int(nc.value),
                                final_rows=int(rows.value), restorations=resto, fallback=fb.bool(), nan_jacobian=nanj.to(torch.int64))


_NATIVE_CACHE = {}


def _native(problem, B, **opts):
    """A cached NativeSolver for this template / batch / options (the last few kept)."""
    key = (bytes(problem.desc()), int(B), tuple(sorted(opts.items())))
    s = _NATIVE_CACHE.get(key)
    if s is None:
        while len(_NATIVE_CACHE) >= 2:
            _NATIVE_CACHE.pop(next(iter(_NATIVE_CACHE)))
        s = _NATIVE_CACHE[key] = NativeSolver(problem, B, **opts)
    return s


# (diagnostics) called with the regular iteration's Newton system and step when set
_DEBUG_NEWTON = None
_DEBUG_TRIAL = None
_DEBUG_EVENT = None


def batch_ipm_solve(problem, X0, mass=None, evaluator: Optional[Callable] = None, tol: float = 1e-8,
                    max_iter: int = 3000, mu_init: float = 0.1, acceptable_tol: float = 1e-6,
                    acceptable_iter: int = 15, max_ls: int = 40, max_soc: int = 4, hessian: str = "exact",
                    fd_step: float = 1e-6, graph: Optional[bool] = None, check_every: int = 4,
                    verbose: int = 0, compact: bool = True, verbose_instance: int = 0,
                    ls_kernel: int = 2, fallback_viol_tol: float = 0.0,
                    nlp_scaling: str = "gradient-based", jacobian_regularization: str = "pivot",
                    watchdog: bool = False, watchdog_trigger: int = 10,
                    watchdog_trial_max: int = 3) -> BatchSolveResult:
    """Solve B instances of `problem`'s template from the starting points X0 [B, n] (torch float64,
    device tensor), per-instance robot masses `mass` [B] (None: the template's).

    evaluator(X [B, n], mass, outputs) -> {name: tensor} for outputs among "f" [B], "grad" [B, n],
    "g" [B, m], "jac" [B, nnz], on X's device; default KernelEvaluator(problem) (the HIP kernel).
    hessian: "exact" (the analytic Lagrangian Hessian, cpl_lagrangian_hessian, for Ground /
    no-environment problems on the device; batched central differences of the Lagrangian gradient
    otherwise), "fd" (always the central differences) or "limited-memory"
    (IPOPT's L-BFGS, 6 pairs).  graph: capture one iteration as a HIP graph (default: on for device tensors).
    max_ls / max_soc: at most this many backtracking trials per iteration (the search also stops below
    IPOPT's alpha_min) / second-order corrections on the first trial (IPOPT max_soc 4).
    ls_kernel (device engine): the whole line search (first trial, its corrections, backtracking) in
    one launch for 47 x 30 systems — 2 (default): always, 1: batches of at most 256 rows, 0: never;
    the same iterates bit for bit.
    fallback_viol_tol (opt-in, default 0 = off; not IPOPT, which returns its last iterate): an instance that stops
    without converging at an iterate violating its original constraints by more than this returns the
    lowest-objective iterate it met that satisfied them to this tolerance (result.fallback).
    nlp_scaling: "gradient-based" (IPOPT's default nlp_scaling_method, which IFOPT's IpoptSolver and the
    reference leave in place: src/CentroidalPlanner.cpp:26-27 sets only derivative_test and
    print_timing_statistics) — at the starting point, the objective is scaled by
    df = max(nlp_scaling_min_value, 100 / max|grad f|) when max|grad f| > 100, and each constraint
    block (the equality rows; the inequality rows) whose largest row gradient exceeds 100 gets
    dc_i = max(nlp_scaling_min_value, 100 * (1 / max(100, max_j |J_ij|))) on every row (gradients over
    the free variables; a NaN entry counts as 0, this solve's NaN policy); the iteration runs on the
    scaled problem (IPOPT's tol applies there), x is not scaled, the returned multipliers are the
    unscaled ones (dc y / df).  "none": no scaling.  The constraint bounds here are 0 or infinite, so
    scaling leaves them unchanged.
    jacobian_regularization: a rank-deficient A (|R_jj| < 1e-10 |R|max): "pivot" (default) adds
    delta_c = 1e-8 mu^0.25 |R|max to R's small pivots; "ipopt" solves IPOPT's [[W, A^T], [A, -delta_c I]]
    (delta_c = 1e-8 mu^0.25) as the augmented system — here and in the engine
    (cpl_solve_options.jacobian_regularization, csrc/cpl_kkt.hip cpl_kkt_aug_kernel).
    watchdog (host path only, opt-in; the engine has none): IPOPT's watchdog procedure
    (BacktrackingLineSearch, watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3) as the
    compiled restatement has it (oracle/cpl_solve_host.c, cplo_set_watchdog): after `watchdog_trigger`
    consecutive shortened steps the iterate and its step are kept; the next iterations take their full
    step judged against the kept iterate's references, a success ends it, the (trial_max + 1)-th failure
    restores the kept iterate and backtracks along its step from alpha_max / 2; a barrier change or the
    restoration phase ends it."""
    if hessian not in ("exact", "fd", "limited-memory"):
        raise ValueError("hessian must be 'exact', 'fd' or 'limited-memory'")
    if nlp_scaling not in ("gradient-based", "none"):
        raise ValueError("nlp_scaling must be 'gradient-based' or 'none'")
    if jacobian_regularization not in ("ipopt", "pivot"):
        raise ValueError("jacobian_regularization must be 'ipopt' or 'pivot'")
    jac_reg = jacobian_regularization == "ipopt"
    use_bfgs = hessian == "limited-memory"
    import torch

    if watchdog and X0.is_cuda:
        raise ValueError("watchdog: the host restatement only (the device engine has no watchdog)")

    if X0.is_cuda:  # device tensors: the native engine (csrc/cpl_solver.hip) with the product callbacks
        if evaluator is not None and not isinstance(evaluator, KernelEvaluator):
            raise ValueError("device solves run the product callbacks (KernelEvaluator); custom evaluators take "
                             "host tensors")
        ns = _native(problem, X0.shape[0], tol=tol, max_iter=max_iter, mu_init=mu_init, acceptable_tol=acceptable_tol,
                     acceptable_iter=acceptable_iter, max_ls=max_ls, max_soc=max_soc, hessian=hessian,
                     fd_step=fd_step, graph=True if graph is None else bool(graph), compact=compact,
                     ls_kernel=ls_kernel, fallback_viol_tol=fallback_viol_tol, nlp_scaling=nlp_scaling,
                     jacobian_regularization=jacobian_regularization)
        r = ns.solve(X0, mass, None if evaluator is None else evaluator.env_tag)
        if evaluator is not None:
            evaluator.calls += r.evaluations
        return r

    # host tensors: this module's restatement, step for step, of the engine's iteration — the checker
    # of the device path over any evaluator's callbacks (tests drive it with the oracle's)
    ev = evaluator if evaluator is not None else KernelEvaluator(problem)
    dev, dt = X0.device, torch.float64
    if graph:
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
    eye_m = torch.eye(m, dtype=dt, device=dev)
    eye_w = torch.eye(nw, dtype=dt, device=dev)
    eye_f = torch.eye(nf, dtype=dt, device=dev)
    fslot = torch.arange(FMAX, device=dev)[None, :]
    fd_cols = torch.arange(nf, device=dev)
    mu_min = min(tol, COMPL_INF_TOL) / (BARRIER_TOL_FACTOR + 1.0)  # IPOPT MonotoneMuUpdate's floor
    xmask = torch.cat([torch.ones(nf, dtype=torch.bool, device=dev), torch.zeros(nI, dtype=torch.bool, device=dev)])

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

    # IPOPT's gradient-based NLP scaling at the starting point (see the docstring): df [B], dc [B, m]
    df = torch.ones(B, dtype=dt, device=dev)
    dc = torch.ones(B, m, dtype=dt, device=dev)
    # (the callbacks at the start point also give the NaN Jacobian entries there: the cone's 0/0)
    n_eval += 1
    o0 = ev(Xbase, Mass, outputs=("jac", "grad"))
    nan_jacobian = torch.isnan(o0["jac"]).sum(1)
    if nlp_scaling == "gradient-based":
        gmax = torch.nan_to_num(o0["grad"][:, free], nan=0.0).abs().amax(1) if nf else zeros_B
        df = torch.where(gmax > SCALING_MAX_GRADIENT,
                         torch.clamp(SCALING_MAX_GRADIENT / torch.where(gmax > 0, gmax, 1.0), min=SCALING_MIN_VALUE),
                         torch.ones_like(gmax))
        if m:
            free_col = torch.zeros(n, dtype=torch.bool, device=dev)
            free_col[free] = True
            aJ = torch.where(free_col[jCol_t], torch.nan_to_num(o0["jac"], nan=0.0).abs(), 0.0)
            rmax = torch.zeros(B, m, dtype=dt, device=dev).scatter_reduce(1, iRow_t.expand(B, -1), aJ, "amax")
            for rows in (torch.as_tensor(np.where(gl_np == gu_np)[0], device=dev), I):
                if rows.numel() == 0:
                    continue
                need = rmax[:, rows].amax(1) > SCALING_MAX_GRADIENT
                d = torch.clamp(SCALING_MAX_GRADIENT * (1.0 / torch.clamp(rmax[:, rows], min=SCALING_MAX_GRADIENT)),
                                min=SCALING_MIN_VALUE)
                dc[:, rows] = torch.where(need[:, None], d, torch.ones_like(d))
    scaled = bool((df != 1.0).any()) or bool((dc != 1.0).any())

    def evaluate_fg(Xe):  # line-search trial points: constraint values and objective only
        nonlocal n_eval
        n_eval += 1
        o = ev(Xe, Mass, outputs=("g", "f"))
        if scaled:
            return {"f": o["f"] * df, "g": o["g"] * dc}
        return {"f": o["f"], "g": o["g"]}

    def evaluate(Xe):
        nonlocal n_eval
        n_eval += 1
        o = ev(Xe, Mass)
        J = torch.zeros(B, m * n, dtype=dt, device=dev)
        J[:, flat_idx] = torch.nan_to_num(o["jac"], nan=0.0)  # a cone at F_t = 0 has a 0/0 Jacobian
        J = J.view(B, m, n)
        if scaled:
            return {"f": o["f"] * df, "grad": o["grad"] * df[:, None], "g": o["g"] * dc, "J": J * dc[:, :, None]}
        return {"f": o["f"], "grad": o["grad"], "g": o["g"], "J": J}

    def y_raw(yv):
        """multipliers of the unscaled callbacks: the scaled problem's Lagrangian df f + (dc y)^T g equals
        df (f + ((dc y) / df)^T g) — the raw Hessian / Lagrangian gradient of the callbacks at these
        multipliers, times df"""
        return (dc * yv) / df[:, None] if scaled else yv

    def unpack(wv):
        Xn = Xbase.clone()
        Xn[:, free] = wv[:, :nf]
        return Xn

    def cons(g, s):
        c = g - gl
        c[:, I] = g[:, I] - s
        return c

    def jac_w(J, mask=None):
        return torch.cat([J[:, :, free], (-P).expand(B, m, nI)], dim=2)

    def barrier(wv, muv):
        dl_ = torch.where(hasL, wv - wl0, torch.ones_like(wv))
        du_ = torch.where(hasU, wu0 - wv, torch.ones_like(wv))
        return -muv * (torch.log(dl_).sum(1) + torch.log(du_).sum(1))

    def fd_hessian(Xc, yv, with_grad=True):
        """Central differences of grad f + J^T y (with_grad False: of J^T y alone — the restoration
        phase's constraint curvature) over x_free."""
        nonlocal n_eval
        h = fd_step * torch.clamp(Xc[:, free].abs(), min=1.0)                       # [B, nf]
        Xp = Xc.unsqueeze(1).repeat(1, 2 * nf, 1)                                   # [B, 2nf, n]
        Xp[:, fd_cols, free] += h
        Xp[:, nf + fd_cols, free] -= h
        n_eval += 1
        o = ev(Xp.view(B * 2 * nf, n), Mass_fd, outputs=("jac", "grad"))
        gL = o["grad"].clone() if with_grad else torch.zeros_like(o["grad"])
        gL.index_add_(1, jCol_t, torch.nan_to_num(o["jac"], nan=0.0) * y_raw(yv).repeat_interleave(2 * nf, 0)[:, iRow_t])
        gL = gL.view(B, 2 * nf, n)[:, :, free]
        H = (gL[:, :nf] - gL[:, nf:]) / (2.0 * h[:, :, None])
        H = 0.5 * (H + H.transpose(1, 2))
        return H * df[:, None, None] if scaled else H

    def hessian_blk(wv, yv, constraints_only=False):
        """Hessian of the Lagrangian over x_free at unpack(wv): the evaluator's analytic one when it has
        one (hessian="exact"), else central differences; constraints_only: of y^T g alone (the
        restoration phase: its objective's curvature is the proximity term, added by the caller)."""
        Xc = unpack(wv)
        if hessian == "exact" and hasattr(ev, "hessian"):
            yr = y_raw(yv)
            Hb = ev.hessian(Xc, yr, free, zero_cost=True) if constraints_only else ev.hessian(Xc, yr, free)
            if Hb is not None:
                return Hb * df[:, None, None] if scaled else Hb
        return fd_hessian(Xc, yv, with_grad=not constraints_only)

    def chol_inertia(K, dwl, mask):
        """Cholesky of K + delta_w I with IPOPT's inertia-correction schedule (first 1e-4, or
        dwl / 3 when the last correction was dwl; x100 / x8 growth); pivots at or below
        _PIVOT_REL max|K_ii| count as zero eigenvalues."""
        nzz = K.shape[1]
        eye_z = torch.eye(nzz, dtype=dt, device=dev)
        piv_tol = _PIVOT_REL * K.diagonal(dim1=1, dim2=2).abs().amax(1)

        def chol(dw_):
            Lf, inf_ = torch.linalg.cholesky_ex(K + dw_[:, None, None] * eye_z)
            if nzz:
                inf_ = torch.where((inf_ == 0) & ((Lf.diagonal(dim1=1, dim2=2) ** 2).amin(1) <= piv_tol),
                                   torch.ones_like(inf_), inf_)
            return Lf, inf_

        delta_w = zeros_B.clone()
        L1, info1 = chol(delta_w)
        for _ in range(64):
            bad = (info1 != 0) & mask
            if not bool(bad.any()):
                break
            first_dw = torch.where(dwl == 0, torch.full_like(delta_w, 1e-4), torch.clamp(dwl / 3.0, min=1e-20))
            grow = delta_w * torch.where(dwl == 0, 100.0, 8.0)
            delta_w = torch.where(bad, torch.where(delta_w == 0, first_dw, grow), delta_w)
            L1n, info1n = chol(delta_w)
            L1 = torch.where(bad[:, None, None], L1n, L1)
            info1 = torch.where(bad, info1n, info1)
        return L1, delta_w

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
        Rd.copy_(torch.where(small, Rd + torch.where(Rd < 0, -dc[:, None], dc[:, None]), Rd))
        Hr = Z.transpose(1, 2) @ M @ Z
        Hr = 0.5 * (Hr + Hr.transpose(1, 2))
        nz = nw - m
        # the inertia test pivots against the full system's M (its largest diagonal entry)
        piv_scale = M.diagonal(dim1=1, dim2=2).abs().amax(1)
        if nz:
            eye_z = torch.eye(nz, dtype=dt)
            piv_tol = _PIVOT_REL * piv_scale

            def chol(dw_):
                Lf, inf_ = torch.linalg.cholesky_ex(Hr + dw_[:, None, None] * eye_z)
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
        else:
            delta_w, L1 = zeros_B.clone(), None
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
        if not (jac_reg and bool(rank_def.any())):
            return dw, dy, delta_w, lambda r2v, mask=None: refined(r1, r2v)[0]
        # IPOPT's regularisation of the rank-deficient systems (jacobian_regularization="ipopt"): the
        # system [[W + dW I, A^T], [A, -delta_c I]], delta_c = 1e-8 mu^0.25, solved as the augmented one
        # in (dw, s): W~ = diag(W, I), A~ = [A, -sqrt(delta_c) I] (full row rank), dW on the W block only
        # — the compiled restatement's kkt_factor with cplo_set_jac_reg (oracle/cpl_solve_host.c)
        idx = torch.nonzero(rank_def).flatten()
        k, na = idx.numel(), nw + m
        sdc = torch.sqrt(1e-8 * mu[idx] ** 0.25)
        Ma = torch.zeros(k, na, na, dtype=dt)
        Ma[:, :nw, :nw] = M[idx]
        Ma[:, nw:, nw:] = torch.eye(m, dtype=dt)
        Aa = torch.cat([A[idx], -sdc[:, None, None] * torch.eye(m, dtype=dt)], 2)
        Qa, Ra_ = torch.linalg.qr(Aa.transpose(1, 2), mode="complete")
        Ya, Za = Qa[:, :, :m], Qa[:, :, m:]
        Ra = Ra_[:, :m, :m]
        Hra = Za.transpose(1, 2) @ Ma @ Za
        Hra = 0.5 * (Hra + Hra.transpose(1, 2))
        Pz = Za[:, :nw, :].transpose(1, 2) @ Za[:, :nw, :]  # dW acts on W only
        piv_tol_a = _PIVOT_REL * Ma.diagonal(dim1=1, dim2=2).abs().amax(1)
        dwl_a = dwl[idx]

        def chol_a(dw_):
            Lf, inf_ = torch.linalg.cholesky_ex(Hra + dw_[:, None, None] * Pz)
            inf_ = torch.where((inf_ == 0) & ((Lf.diagonal(dim1=1, dim2=2) ** 2).amin(1) <= piv_tol_a),
                               torch.ones_like(inf_), inf_)
            return Lf, inf_

        dwa = torch.zeros(k, dtype=dt)
        La, infa = chol_a(dwa)
        for _ in range(64):
            bad = infa != 0
            if not bool(bad.any()):
                break
            first_dw = torch.where(dwl_a == 0, torch.full_like(dwa, 1e-4), torch.clamp(dwl_a / 3.0, min=1e-20))
            grow = dwa * torch.where(dwl_a == 0, 100.0, 8.0)
            dwa = torch.where(bad, torch.where(dwa == 0, first_dw, grow), dwa)
            Ln, infn = chol_a(dwa)
            La = torch.where(bad[:, None, None], Ln, La)
            infa = torch.where(bad, infn, infa)
        Mwa = Ma.clone()
        Mwa[:, :nw, :nw] += dwa[:, None, None] * eye_w

        def solve_a(q1, q2):
            py = torch.linalg.solve_triangular(Ra.transpose(1, 2), q2.unsqueeze(2), upper=False)
            d = Ya @ py
            pz = torch.cholesky_solve(Za.transpose(1, 2) @ (q1.unsqueeze(2) - Mwa @ d), La)
            d = d + Za @ pz
            dy_ = torch.linalg.solve_triangular(Ra, Ya.transpose(1, 2) @ (q1.unsqueeze(2) - Mwa @ d), upper=True)
            return d.squeeze(2), dy_.squeeze(2)

        def refined_a(q1, q2):
            q1a = torch.cat([q1, torch.zeros(k, m, dtype=dt)], 1)
            d1, d2 = solve_a(q1a, q2)
            e1 = q1a - (Mwa @ d1.unsqueeze(2)).squeeze(2) - (Aa.transpose(1, 2) @ d2.unsqueeze(2)).squeeze(2)
            e2 = q2 - (Aa @ d1.unsqueeze(2)).squeeze(2)
            c1, c2 = solve_a(e1, e2)
            return (d1 + c1)[:, :nw], d2 + c2

        dwr, dyr = refined_a(r1[idx], r2[idx])
        dw, dy, delta_w = dw.clone(), dy.clone(), delta_w.clone()
        dw[idx], dy[idx], delta_w[idx] = dwr, dyr, dwa

        def solve_primal(r2v, mask=None):
            d = refined(r1, r2v)[0].clone()
            d[idx] = refined_a(r1[idx], r2v[idx])[0]
            return d

        return dw, dy, delta_w, solve_primal

    def kkt_qd(W, A, Dinv, r1, r2, dwl, mask):
        """The restoration phase's Newton system after p and n are eliminated (as IPOPT's
        AugRestoSystemSolver reduces it): [[W, A^T], [A, -D]] [dw; dy] = [r1; r2], D = 1 / Dinv > 0
        diagonal.  The primal Schur complement K = W + A^T Dinv A is factorised with the inertia
        correction (the full system has the right inertia iff K is positive definite);
        dw = K^-1 (r1 + A^T Dinv r2), dy = Dinv (A dw - r2)."""
        K = W + A.transpose(1, 2) @ (Dinv[:, :, None] * A)
        K = 0.5 * (K + K.transpose(1, 2))
        L1, delta_w = chol_inertia(K, dwl, mask)
        rhs = r1 + (A.transpose(1, 2) @ (Dinv * r2).unsqueeze(2)).squeeze(2)
        dw = torch.cholesky_solve(rhs.unsqueeze(2), L1).squeeze(2)
        dy = Dinv * ((A @ dw.unsqueeze(2)).squeeze(2) - r2)
        return dw, dy, delta_w

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
        return {"A": A_, "gw": gw, "c": c_, "d_inf": d_inf, "c_inf": c_inf, "base": base, "cl": cl, "cu": cu,
                "sc": sc, "err0": torch.maximum(base, torch.maximum(cl.amax(1), cu.amax(1)) / sc)}

    def err_mu(E, muv):
        comp_mu = torch.maximum((E["cl"] - torch.where(hasL, muv[:, None], 0.0)).abs().amax(1),
                                (E["cu"] - torch.where(hasU, muv[:, None], 0.0)).abs().amax(1))
        return torch.maximum(E["base"], comp_mu / E["sc"])

    def pd_error(o, wv, yv, zl, zu, muv):
        """IPOPT's primal-dual system error of the barrier problem (1-norms of the dual residual, the
        constraint residual and the mu-complementarity; the soft restoration phase's measure)."""
        A_ = jac_w(o["J"])
        gw = torch.cat([o["grad"][:, free], zeros_I], 1)
        dual = gw + (A_.transpose(1, 2) @ yv.unsqueeze(2)).squeeze(2) - zl + zu
        c_ = cons(o["g"], wv[:, nf:])
        cl = torch.where(hasL, (wv - wl0) * zl - muv[:, None], torch.zeros_like(wv))
        cu = torch.where(hasU, (wu0 - wv) * zu - muv[:, None], torch.zeros_like(wv))
        return dual.abs().sum(1) + c_.abs().sum(1) + cl.abs().sum(1) + cu.abs().sum(1)

    def reset_filter(mask, ft, fp, fc):
        return (torch.where(mask[:, None], torch.full_like(ft, float("inf")), ft),
                torch.where(mask[:, None], torch.full_like(fp, float("inf")), fp),
                torch.where(mask, torch.zeros_like(fc), fc))

    def augment_filter(mask, ft, fp, fc, th, ph):
        """IPOPT's AugmentFilter: the entry ((1 - gamma_theta) theta, phi - gamma_phi theta) into the ring."""
        fi = fslot == torch.remainder(fc, FMAX)[:, None]
        ft = torch.where(mask[:, None] & fi, ((1.0 - GAMMA_TH) * th)[:, None], ft)
        fp = torch.where(mask[:, None] & fi, (ph - GAMMA_PHI * th)[:, None], fp)
        return ft, fp, fc + mask.to(fc.dtype)

    def max_step(v, dv, lo_mask, lo, tau):
        r = torch.where(lo_mask & (dv < 0), -tau[:, None] * (v - lo) / torch.where(dv < 0, dv, -1.0),
                        torch.full_like(v, float("inf")))
        return torch.clamp(r.amin(1), max=1.0)

    def alpha_min_of(theta_k, gd, theta_min):
        """IPOPT FilterLSAcceptor::CalculateAlphaMin: the smallest trial step before the line search
        gives up (alpha_min_frac 0.05)."""
        ngd = torch.where(gd < 0, -gd, torch.ones_like(gd))
        a = torch.minimum(torch.full_like(gd, GAMMA_TH), GAMMA_PHI * theta_k / ngd)
        a = torch.where(theta_k <= theta_min, torch.minimum(a, DELTA_SW * theta_k ** S_TH / ngd ** S_PHI), a)
        return ALPHA_MIN_FRAC * torch.where(gd < 0, a, torch.full_like(gd, GAMMA_TH))

    def acceptable(th, ph, theta_k, phi_k, gd, al, switch_ok, theta_max, ft, fp, from_resto=False):
        """IPOPT FilterLSAcceptor::CheckAcceptabilityOfTrialPoint: theta_max, then Armijo on the
        barrier objective for an f-type step (switching condition) at a reference point with
        theta_k <= theta_min, or the sufficient decrease of theta or phi against the current iterate
        (with the obj_max_inc guard), then the filter (entries stored with their margins).  switch_ok:
        theta_k <= theta_min (gd < 0 is tested here).  Returns (ok, h_type): h_type = the step augments
        the filter — UpdateForNextIteration: unless IsFtype (the switching condition alone, no
        theta_min term) and Armijo hold."""
        fin = torch.isfinite(ph) & torch.isfinite(th)
        in_filter = ((th[:, None] <= ft) | (ph[:, None] <= fp)).all(1)
        is_ftype = (gd < 0) & (al * torch.where(gd < 0, -gd, torch.zeros_like(gd)) ** S_PHI > DELTA_SW * theta_k ** S_TH)
        ftype = is_ftype & switch_ok
        # IPOPT's Compare_le(lhs, rhs, base): lhs - rhs <= 10 eps |base| (round-off of the reference values)
        ro_p, ro_t = 10.0 * EPS * phi_k.abs(), 10.0 * EPS * theta_k.abs()
        armijo = (ph - phi_k) - ETA_PHI * al * gd <= ro_p
        suff = (th - (1.0 - GAMMA_TH) * theta_k <= ro_t) | ((ph - phi_k) - (-GAMMA_PHI * theta_k) <= ro_p)
        if not from_resto:  # obj_max_inc = 5: the barrier objective may not jump by 5 orders of magnitude
            base = torch.where(phi_k.abs() > 10.0, torch.log10(phi_k.abs().clamp(min=1e-300)), torch.ones_like(phi_k))
            inc = ph - phi_k
            big = (inc > 0) & (torch.log10(inc.clamp(min=1e-300)) > OBJ_MAX_INC + base)
            suff = suff & ~big
            armijo = armijo & ~big
        ok = fin & (th <= theta_max) & in_filter & torch.where(ftype, armijo, suff)
        return ok, ~(is_ftype & armijo)

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

    zB = lambda: zeros_B.clone()  # noqa: E731
    zBm = lambda: torch.zeros(B, m, dtype=dt, device=dev)  # noqa: E731
    zBw = lambda: torch.zeros(B, nw, dtype=dt, device=dev)  # noqa: E731
    bool_B = lambda: torch.zeros(B, dtype=torch.bool, device=dev)  # noqa: E731
    # persistent state: the iteration reads these and writes them back in place
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
        "dwl": zB(),
        "f": cur0["f"].clone(), "grad": cur0["grad"].clone(), "g": cur0["g"].clone(), "J": cur0["J"].clone(),
        "d_inf": zB(),
        "tiny_last": bool_B(), "tiny_flag": bool_B(),
        "in_soft": bool_B(), "soft_cnt": torch.zeros(B, dtype=torch.int64, device=dev),
        "Hq": eye_f.repeat(B, 1, 1) if use_bfgs else None,
        "lm_s": torch.zeros(B, LM_HIST, nf, dtype=dt, device=dev) if use_bfgs else None,
        "lm_y": torch.zeros(B, LM_HIST, nf, dtype=dt, device=dev) if use_bfgs else None,
        "lm_cnt": torch.zeros(B, dtype=torch.int64, device=dev),
        "lm_skip": torch.zeros(B, dtype=torch.int64, device=dev),
        # restoration phase (IPOPT's MinC_1NrmRestorationPhase): per instance, a second interior-point
        # problem in the same lock-step iteration
        "resto": bool_B(), "wR": zBw(), "p": zBm(), "n": zBm(), "zp": zBm(), "zn": zBm(), "zLR": zBw(),
        "zUR": zBw(), "muR": zB(), "ftR": torch.full((B, FMAX), float("inf"), dtype=dt, device=dev),
        "fpR": torch.full((B, FMAX), float("inf"), dtype=dt, device=dev),
        "fcR": torch.zeros(B, dtype=torch.int64, device=dev), "th_o0": zB(), "ph_o0": zB(), "dwlR": zB(),
        "thmaxR": zB(), "thminR": zB(), "n_resto": torch.zeros(B, dtype=torch.int64, device=dev),
        "resto_tight": bool_B(),
        # the best iterate feasible to fallback_viol_tol (lowest f): the fallback result of a solve that
        # stops without converging at an infeasible iterate (not IPOPT)
        "best_w": zBw(), "best_f": torch.full((B,), float("inf"), dtype=dt, device=dev),
        # IPOPT's backup acceptable point (BacktrackingLineSearch::StoreAcceptablePoint): the last
        # regular iterate at the acceptable level, restored when the restoration phase fails
        "acc_w": zBw(), "acc_y": zBm(), "acc_zL": zBw(), "acc_zU": zBw(), "has_acc": bool_B(),
    }
    if watchdog:  # IPOPT's watchdog: its state, the kept iterate, its step, evaluation and references
        S.update({"in_wd": bool_B(), "wd_cnt": torch.zeros(B, dtype=torch.int64, device=dev),
                  "wd_trial": torch.zeros(B, dtype=torch.int64, device=dev), "wd_w": zBw(), "wd_y": zBm(),
                  "wd_zL": zBw(), "wd_zU": zBw(), "wd_dw": zBw(), "wd_dy": zBm(), "wd_dzL": zBw(), "wd_dzU": zBw(),
                  "wd_f": torch.zeros_like(S["f"]), "wd_grad": torch.zeros_like(S["grad"]),
                  "wd_g": torch.zeros_like(S["g"]), "wd_J": torch.zeros_like(S["J"]), "wd_th": zB(), "wd_ph": zB(),
                  "wd_gd": zB(), "wd_alpha": zB()})

    def orig_violation(g):
        """max violation of g against the original constraint bounds (NaN: infinite); g is the scaled
        problem's dc g when the solve is scaled, so the original constraints' values are g / dc."""
        if not m:
            return zeros_B
        if scaled:
            g = g / dc
        v = torch.clamp(torch.maximum(gl - g, g - gu), min=0.0).amax(1)
        return torch.where(torch.isnan(g).any(1), torch.full_like(v, float("inf")), v)

    def track_best():
        v = orig_violation(S["g"])
        upd = S["active"] & (v <= fallback_viol_tol) & (S["f"] < S["best_f"])
        S["best_w"].copy_(torch.where(upd[:, None], S["w"], S["best_w"]))
        S["best_f"].copy_(torch.where(upd, S["f"], S["best_f"]))

    def check(E, mask):
        """Convergence test at the current iterate of the instances in `mask`; updates status /
        active / acc."""
        active = S["active"]
        e0 = E["err0"]
        act = active & mask
        done_now = act & (e0 <= tol)
        acc = torch.where(act & (e0 <= acceptable_tol), S["acc"] + 1, torch.where(act, 0, S["acc"]))
        acc_now = act & ~done_now & (acc >= acceptable_iter)
        status = torch.where(done_now, torch.full_like(S["status"], STATUS_OPTIMAL),
                             torch.where(acc_now, torch.full_like(S["status"], STATUS_ACCEPTABLE), S["status"]))
        S["acc"].copy_(acc)
        S["status"].copy_(status)
        S["active"].copy_(active & ~done_now & ~acc_now)
        S["d_inf"].copy_(torch.where(mask, E["d_inf"], S["d_inf"]))

    def lbfgs_reset(mask):
        if use_bfgs:
            S["lm_skip"].copy_(torch.where(mask, 0, S["lm_skip"]))
            S["lm_cnt"].copy_(torch.where(mask, 0, S["lm_cnt"]))
            S["Hq"].copy_(torch.where(mask[:, None, None], eye_f.expand_as(S["Hq"]), S["Hq"]))

    def lbfgs_update(active, sk, new, cur, y_new, with_grad=True):
        """IPOPT's LimMemQuasiNewtonUpdater with IFOPT's defaults (bfgs, max_history 6, scalar1,
        init_val 1 in [1e-8, 1e8], max_skipping 2) — the device's k_lbfgs (csrc/cpl_solver.hip).
        with_grad False: the pair from J^T y alone (the restoration phase's model of its
        constraint curvature; its proximity term's Hessian is exact and added separately)."""
        JTy_new = (new["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
        JTy_old = (cur["J"].transpose(1, 2) @ y_new.unsqueeze(2)).squeeze(2)
        if with_grad:
            yk = (new["grad"] + JTy_new)[:, free] - (cur["grad"] + JTy_old)[:, free]
        else:
            yk = (0.0 + JTy_new)[:, free] - (0.0 + JTy_old)[:, free]
        sy, ss, yy = (sk * yk).sum(1), (sk * sk).sum(1), (yk * yk).sum(1)
        take = active & (sy > math.sqrt(EPS) * ss.sqrt() * yy.sqrt())
        skip = active & ~take
        skipped = torch.where(skip, S["lm_skip"] + 1, torch.zeros_like(S["lm_skip"]))
        reset = skip & (skipped > LM_MAX_SKIP)
        S["lm_skip"].copy_(torch.where(active, torch.where(reset, torch.zeros_like(skipped), skipped), S["lm_skip"]))
        # memory: a full one shifts down by one (the oldest pair dropped), the new pair appended
        cnt = S["lm_cnt"]
        full = (cnt == LM_HIST)[:, None, None]
        Ps = torch.where(full, S["lm_s"].roll(-1, 1), S["lm_s"])
        Py = torch.where(full, S["lm_y"].roll(-1, 1), S["lm_y"])
        last = torch.clamp(cnt, max=LM_HIST - 1)
        slot = (torch.arange(LM_HIST, device=dev)[None, :] == last[:, None])[:, :, None]
        Ps = torch.where(slot, sk[:, None, :], Ps)
        Py = torch.where(slot, yk[:, None, :], Py)
        nc = last + 1
        S["lm_s"].copy_(torch.where(take[:, None, None], Ps, S["lm_s"]))
        S["lm_y"].copy_(torch.where(take[:, None, None], Py, S["lm_y"]))
        S["lm_cnt"].copy_(torch.where(take, nc, torch.where(reset, torch.zeros_like(cnt), cnt)))
        # the dense model rebuilt from sigma I by the recursion over the stored pairs, oldest first (the
        # device's k_lbfgs evaluates the same model with the recursion unrolled onto vectors: equal up to
        # rounding)
        sigma = torch.clamp(sy / torch.where(ss > 0, ss, 1.0), min=1e-8, max=1e8)
        H = sigma[:, None, None] * eye_f
        for j in range(LM_HIST):
            sj, yj = Ps[:, j], Py[:, j]
            Hs = (H @ sj.unsqueeze(2)).squeeze(2)
            sHs, sjy = (sj * Hs).sum(1), (sj * yj).sum(1)
            ok = (j < nc) & (sHs > 0)
            Hn = (H - Hs.unsqueeze(2) * Hs.unsqueeze(1) / torch.where(ok, sHs, 1.0)[:, None, None]) + \
                yj.unsqueeze(2) * yj.unsqueeze(1) / torch.where(ok, sjy, 1.0)[:, None, None]
            H = torch.where(ok[:, None, None], Hn, H)
        Hq = torch.where(take[:, None, None], H, S["Hq"])
        S["Hq"].copy_(torch.where(reset[:, None, None], eye_f.expand_as(Hq), Hq))

    def trial_ls(wv, d, al, mask, st):
        """A trial point w + al d for the instances in mask (others: their line-search state's point)."""
        wt_ = wv + al[:, None] * d
        return wt_, evaluate_fg(unpack(torch.where(mask[:, None], wt_, st["w"])))

    def take(st, mask, wt, o, al, aug_mask, extra=None):
        st["f"] = torch.where(mask, o["f"], st["f"])
        st["g"] = torch.where(mask[:, None], o["g"], st["g"])
        st["w"] = torch.where(mask[:, None], wt, st["w"])
        st["alpha"] = torch.where(mask, al, st["alpha"])
        st["aug"] = torch.where(mask, aug_mask, st["aug"])
        st["found"] = st["found"] | mask
        st["searching"] = st["searching"] & ~mask
        if extra is not None:
            for k, v in extra.items():
                st[k] = torch.where(mask.view(-1, *([1] * (v.dim() - 1))), v, st[k])

    # ------------------------------------------------------------------------------------------
    def regular_step(E, act):
        """One IPOPT iteration of the instances in `act` (not in the restoration phase)."""
        w, y, zL, zU, mu = S["w"], S["y"], S["zL"], S["zU"], S["mu"].clone()
        cur = {"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}
        A, gradw, c = E["A"], E["gw"], E["c"]
        # IPOPT stores the current iterate as the backup acceptable point when it is at the
        # acceptable level (FindAcceptableTrialPoint: CurrentIsAcceptable -> StoreAcceptablePoint)
        store = act & (E["err0"] <= acceptable_tol)
        for k, v in (("acc_w", w), ("acc_y", y), ("acc_zL", zL), ("acc_zU", zU)):
            S[k].copy_(torch.where(store[:, None], v, S[k]))
        S["has_acc"].copy_(S["has_acc"] | store)
        # ---- monotone barrier update (IPOPT MonotoneMuUpdate with mu_allow_fast_monotone_decrease: as
        # long as the barrier problem is solved to kappa_eps mu, or once after two tiny steps), the
        # filter reset where mu changed
        ft, fp, fc = S["filt_t"], S["filt_p"], S["fcount"]
        force = S["tiny_flag"] & act
        for r in range(MU_ROUNDS):
            upd = act & ((err_mu(E, mu) <= BARRIER_TOL_FACTOR * mu) | (force if r == 0 else False)) & (mu > mu_min)
            mu = torch.where(upd, torch.clamp(torch.minimum(0.2 * mu, mu ** 1.5), min=mu_min), mu)
            ft, fp, fc = reset_filter(upd, ft, fp, fc)
            # IPOPT's BacktrackingLineSearch::Reset (MonotoneMuUpdate calls it when mu changes): the
            # filter reset above and the end of the soft restoration phase (and of the watchdog)
            S["in_soft"].copy_(S["in_soft"] & ~upd)
            if watchdog:
                S["in_wd"].copy_(S["in_wd"] & ~upd)
                S["wd_cnt"].copy_(torch.where(upd, 0, S["wd_cnt"]))
        tau = torch.clamp(1.0 - mu, min=0.99)

        def primal_step(d):  # fraction to the boundary along d from w
            return torch.minimum(max_step(w, d, hasL, wl0, tau), max_step(-w, -d, hasU, -wu0, tau))

        Hblk = S["Hq"] if use_bfgs else hessian_blk(w, y)
        dl = torch.where(hasL, w - wl0, torch.ones_like(w))
        du = torch.where(hasU, wu0 - w, torch.ones_like(w))
        Sig = torch.where(hasL, zL / dl, torch.zeros_like(w)) + torch.where(hasU, zU / du, torch.zeros_like(w))
        gphi = gradw - torch.where(hasL, mu[:, None] / dl, torch.zeros_like(w)) + \
            torch.where(hasU, mu[:, None] / du, torch.zeros_like(w))
        r1 = -(gphi + (A.transpose(1, 2) @ y.unsqueeze(2)).squeeze(2))
        r2 = -c
        M = torch.diag_embed(Sig)
        M[:, :nf, :nf] += Hblk
        theta_k = c.abs().sum(1)
        phi_k = cur["f"] + barrier(w, mu)
        dw, dy, delta_w, solve_primal = kkt_host(M, A, r1, r2, mu, S["dwl"], act)
        if _DEBUG_NEWTON is not None:  # (diagnostics: scripts/solve_divergence.py)
            _DEBUG_NEWTON(dict(M=M, A=A, r1=r1, r2=r2, dw=dw, dy=dy, w=w, y=y, it=it_run))
        dwl = torch.where(act, delta_w, S["dwl"])
        dzL = torch.where(hasL, mu[:, None] / dl - zL - zL / dl * dw, torch.zeros_like(w))
        dzU = torch.where(hasU, mu[:, None] / du - zU + zU / du * dw, torch.zeros_like(w))
        a_max = primal_step(dw)
        a_z = torch.minimum(max_step(zL, dzL, hasL, 0.0, tau), max_step(zU, dzU, hasU, 0.0, tau))
        gd = (gphi * dw).sum(1)
        switch_ok = theta_k <= theta_min
        # IPOPT DetectTinyStep: the step is below 10 eps relative in every primal component, the
        # multiplier step below 1e-2, the point feasible to 1e-4: taken whole without a line search;
        # two in a row force the next barrier decrease
        tiny = act & ((dw.abs() / (1.0 + w.abs())).amax(1) < TINY_STEP_TOL) & \
            (dy.abs().amax(1) < TINY_STEP_Y_TOL) & (E["c_inf"] < 1e-4)
        S["tiny_flag"].copy_(torch.where(act, tiny & S["tiny_last"], S["tiny_flag"]))
        S["tiny_last"].copy_(torch.where(act, tiny & ~S["tiny_last"], S["tiny_last"]))
        a_min = alpha_min_of(theta_k, gd, theta_min)
        soft_now = act & S["in_soft"] & ~tiny

        # ---- IPOPT's backtracking filter line search: trials alpha_max, alpha_max / 2, ... while
        # alpha > alpha_min (at most max_ls), up to max_soc second-order corrections on the first;
        # in IPOPT's soft restoration phase the backtracking is skipped: only the full primal-dual
        # step is tried (at most max_soft_resto_iters iterations in a row)
        S["soft_cnt"].copy_(S["soft_cnt"] + soft_now.to(torch.int64))
        st = {"searching": act & ~tiny & ~soft_now, "found": bool_B(), "f": cur["f"].clone(),
              "g": cur["g"].clone(), "w": w.clone(), "alpha": zB(), "aug": bool_B()}

        def judge_take(wt_, o_, al, extra_mask=None):
            th_ = cons(o_["g"], wt_[:, nf:]).abs().sum(1)
            ph_ = o_["f"] + barrier(wt_, mu)
            ok_, h_ = acceptable(th_, ph_, theta_k, phi_k, gd, al, switch_ok, theta_max, ft, fp)
            sel = st["searching"] & ok_
            if extra_mask is not None:
                sel = sel & extra_mask
            if _DEBUG_TRIAL is not None:  # (diagnostics)
                _DEBUG_TRIAL(dict(alpha=al, th=th_, ph=ph_, ok=ok_, sel=sel, soc=extra_mask is not None, a_min=a_min,
                                  theta_k=theta_k, phi_k=phi_k, gd=gd))
            take(st, sel, wt_, o_, al, h_)
            return ok_, th_

        R = bool_B()  # (watchdog: the instances whose kept iterate is restored this iteration)
        if watchdog and bool((S["in_wd"] & st["searching"]).any()):
            # IPOPT's watchdog iteration: one trial, the full step, judged against the kept iterate's
            # references; acceptable ends the watchdog, else the step is taken anyway up to trial_max
            # times, after which the kept iterate is restored (StopWatchDog) and searched along its step
            wd = S["in_wd"] & st["searching"]
            theta_k = torch.where(wd, S["wd_th"], theta_k)
            phi_k = torch.where(wd, S["wd_ph"], phi_k)
            gd = torch.where(wd, S["wd_gd"], gd)
            switch_ok = torch.where(wd, S["wd_th"] <= theta_min, switch_ok)
            wt, o = trial_ls(w, dw, a_max, wd, st)
            th_ = cons(o["g"], wt[:, nf:]).abs().sum(1)
            ok_, h_ = acceptable(th_, o["f"] + barrier(wt, mu), theta_k, phi_k, gd, S["wd_alpha"], switch_ok,
                                 theta_max, ft, fp)
            trial = torch.where(wd & ~ok_, S["wd_trial"] + 1, S["wd_trial"])
            S["wd_trial"].copy_(trial)
            tk = wd & (ok_ | (trial <= watchdog_trial_max))
            take(st, tk, wt, o, a_max, h_)
            st["searching"] = st["searching"] & ~wd
            if _DEBUG_EVENT is not None:  # (diagnostics / tests)
                _DEBUG_EVENT("watchdog_success", wd & ok_)
                _DEBUG_EVENT("watchdog_restore", wd & ~tk)
            S["in_wd"].copy_(S["in_wd"] & ~(wd & ok_))
            R = wd & ~tk
            if bool(R.any()):
                S["in_wd"].copy_(S["in_wd"] & ~R)
                S["wd_cnt"].copy_(torch.where(R, 0, S["wd_cnt"]))
                for k in ("w", "y", "zL", "zU", "f", "grad", "g", "J"):  # (w, y, zL, zU, cur alias these)
                    v = S[k]
                    v.copy_(torch.where(R.view(-1, *([1] * (v.dim() - 1))), S["wd_" + k], v))
                dw = torch.where(R[:, None], S["wd_dw"], dw)
                dy = torch.where(R[:, None], S["wd_dy"], dy)
                dzL = torch.where(R[:, None], S["wd_dzL"], dzL)
                dzU = torch.where(R[:, None], S["wd_dzU"], dzU)
                E = errors(cur, w, y, zL, zU)
                A, gradw, c = E["A"], E["gw"], E["c"]
                a_max = torch.where(R, primal_step(dw), a_max)
                a_z = torch.where(R, torch.minimum(max_step(zL, dzL, hasL, 0.0, tau), max_step(zU, dzU, hasU, 0.0, tau)),
                                  a_z)
                a_min = torch.where(R, alpha_min_of(theta_k, gd, theta_min), a_min)
                st["w"] = torch.where(R[:, None], w, st["w"])
                st["f"] = torch.where(R, cur["f"], st["f"])
                st["g"] = torch.where(R[:, None], cur["g"], st["g"])
                st["searching"] = st["searching"] | (R & (0.5 * a_max > a_min))
        alpha = torch.where(R, 0.5 * a_max, a_max)
        n_steps = R.to(torch.int64)  # (the watchdog's shortened-step count: halvings before acceptance)
        for ls in range(max(1, max_ls)):
            if watchdog:  # a restored instance searches from its second trial on (no full step, no SOC)
                st["searching"] = st["searching"] & ~(R & (ls >= max(1, max_ls) - 1))
            if not bool(st["searching"].any()):
                break
            wt, o = trial_ls(w, dw, alpha, st["searching"], st)
            ok, th = judge_take(wt, o, alpha)
            if ls == 0:
                if max_soc > 0:
                    soc = st["searching"] & (th >= theta_k) & ~R
                    c_soc, a_soc, th_old = c, alpha, th
                    ct = cons(o["g"], wt[:, nf:])
                    for _ in range(max_soc):
                        if not bool(soc.any()):
                            break
                        c_soc = a_soc[:, None] * c_soc + ct
                        dws = solve_primal(-c_soc, soc)
                        a_soc = primal_step(dws)
                        ws, os_ = trial_ls(w, dws, a_soc, soc, st)
                        oks, ths = judge_take(ws, os_, alpha, soc)
                        soc = soc & ~oks & (ths <= KAPPA_SOC * th_old)  # kappa_soc = 0.99
                        th_old = ths
                        ct = cons(os_["g"], ws[:, nf:])
            alpha = torch.where(st["searching"], 0.5 * alpha, alpha)
            n_steps = n_steps + st["searching"].to(torch.int64)
            st["searching"] = st["searching"] & (alpha > a_min)  # IPOPT: the next trial only above alpha_min
        if watchdog:  # the shortened-step count; the watchdog starts at this iterate and its step
            fnd = st["found"]
            S["wd_cnt"].copy_(torch.where(fnd, torch.where(n_steps == 0, 0, S["wd_cnt"] + 1), S["wd_cnt"]))
            start = fnd & ~S["in_wd"] & ~soft_now & (S["wd_cnt"] >= watchdog_trigger)
            if bool(start.any()):
                if _DEBUG_EVENT is not None:
                    _DEBUG_EVENT("watchdog_start", start.clone())
                for k, v in (("w", w), ("y", y), ("zL", zL), ("zU", zU), ("dw", dw), ("dy", dy), ("dzL", dzL),
                             ("dzU", dzU), ("f", cur["f"]), ("grad", cur["grad"]), ("g", cur["g"]), ("J", cur["J"]),
                             ("th", theta_k), ("ph", phi_k), ("gd", gd), ("alpha", a_max)):
                    S["wd_" + k].copy_(torch.where(start.view(-1, *([1] * (v.dim() - 1))), v, S["wd_" + k]))
                S["in_wd"].copy_(S["in_wd"] | start)
                S["wd_trial"].copy_(torch.where(start, 0, S["wd_trial"]))
        # tiny steps: the whole fraction-to-the-boundary step
        w_tiny = w + a_max[:, None] * dw
        st["w"] = torch.where(tiny[:, None], w_tiny, st["w"])
        st["alpha"] = torch.where(tiny, a_max, st["alpha"])
        # ---- IPOPT's soft restoration step (TrySoftRestoStep): when the backtracking failed (or in the
        # soft restoration phase) the full primal-dual step alpha = min(alpha_primal_max, alpha_dual_max)
        # for every variable, taken when the original filter / current iterate accept it, or when it
        # cuts the primal-dual error of the barrier problem (1-norms) by soft_resto_pderror_reduction_factor
        bt_failed = act & ~tiny & ~soft_now & ~st["found"]
        soft_try = (soft_now & (S["soft_cnt"] <= MAX_SOFT_RESTO)) | bt_failed
        a_soft = torch.minimum(a_max, a_z)
        soft_ok = bool_B()
        if bool(soft_try.any()):
            ws = w + a_soft[:, None] * dw
            os_ = evaluate(unpack(torch.where(soft_try[:, None], ws, w)))
            th_s = cons(os_["g"], ws[:, nf:]).abs().sum(1)
            ph_s = os_["f"] + barrier(ws, mu)
            orig_ok, _ = acceptable(th_s, ph_s, theta_k, phi_k, gd, zB(), switch_ok, theta_max, ft, fp)
            ys = y + a_soft[:, None] * dy
            zLs = torch.where(hasL, zL + a_soft[:, None] * dzL, zL)
            zUs = torch.where(hasU, zU + a_soft[:, None] * dzU, zU)
            fin_s = torch.isfinite(th_s) & torch.isfinite(ph_s)
            better = pd_error(os_, ws, ys, zLs, zUs, mu) <= SOFT_RESTO_FACTOR * pd_error(cur, w, y, zL, zU, mu)
            soft_ok = soft_try & fin_s & (orig_ok | better)
            take(st, soft_ok, ws, os_, a_soft, bool_B())
            left = soft_ok & orig_ok  # the original criterion holds: the soft phase ends
            S["in_soft"].copy_(torch.where(left, False, torch.where(soft_ok, True, S["in_soft"])))
            S["soft_cnt"].copy_(torch.where(left | (soft_ok & ~soft_now), 0, S["soft_cnt"]))
        failed = act & ~tiny & ~st["found"]  # -> the restoration phase
        # IPOPT calls no restoration phase at an acceptable point (BacktrackingLineSearch: "Restoration
        # phase called at acceptable point" -> STOP_AT_ACCEPTABLE_POINT): the solve ends there
        at_acc = failed & (E["err0"] <= acceptable_tol)
        # nor at an almost feasible point (theta <= 1e-2 tol): the backup acceptable point is restored
        # and the solve stops there as acceptable (RestoreAcceptablePoint), or without one it ends as a
        # restoration failure ("Restoration phase called, but point is almost feasible")
        near = failed & ~at_acc & (theta_k <= ALMOST_FEASIBLE * tol)
        back = near & S["has_acc"]
        if _DEBUG_EVENT is not None and bool(back.any()):  # (diagnostics / tests)
            _DEBUG_EVENT("restore_acceptable_point", back.clone())
        for k, kk in (("w", "acc_w"), ("y", "acc_y"), ("zL", "acc_zL"), ("zU", "acc_zU")):
            S[k].copy_(torch.where(back[:, None], S[kk], S[k]))
        at_acc = at_acc | back
        stop = at_acc | near
        act_it = act & ~stop  # the instances whose iteration counts
        if bool(stop.any()):
            S["status"].copy_(torch.where(at_acc, STATUS_ACCEPTABLE, torch.where(near, STATUS_RESTO_FAILED,
                                                                                   S["status"])))
            S["active"].copy_(S["active"] & ~stop)
            failed = failed & ~stop
        S["in_soft"].copy_(S["in_soft"] & ~failed)
        S["soft_cnt"].copy_(torch.where(failed, 0, S["soft_cnt"]))
        moved = act_it & ~failed
        w_new = st["w"]
        al = st["alpha"]
        a_z = torch.where(soft_ok, a_soft, a_z)  # the soft step moves the bound multipliers by alpha too
        # the accepted points with their derivatives: one full evaluation (trials carried f and g only)
        new = evaluate(unpack(w_new))
        addm = st["aug"] & moved
        ft, fp, fc = augment_filter(addm, ft, fp, fc, theta_k, phi_k)

        # ---- accept: primal, multipliers, bound multipliers (kappa_Sigma safeguard)
        mv = moved[:, None]
        y_new = torch.where(mv, y + al[:, None] * dy, y)
        zL_new = torch.where(mv & hasL, zL + a_z[:, None] * dzL, zL)
        zU_new = torch.where(mv & hasU, zU + a_z[:, None] * dzU, zU)
        dln = torch.where(hasL, w_new - wl0, torch.ones_like(w))
        dun = torch.where(hasU, wu0 - w_new, torch.ones_like(w))
        zL_new = torch.where(mv & hasL, torch.minimum(torch.maximum(zL_new, mu[:, None] / (KAPPA_SIGMA * dln)),
                                                      KAPPA_SIGMA * mu[:, None] / dln), zL_new)
        zU_new = torch.where(mv & hasU, torch.minimum(torch.maximum(zU_new, mu[:, None] / (KAPPA_SIGMA * dun)),
                                                      KAPPA_SIGMA * mu[:, None] / dun), zU_new)
        if use_bfgs:  # IPOPT's limited-memory BFGS over x_free (both Lagrangian gradients at the new y)
            lbfgs_update(moved, (w_new - w)[:, :nf], new, cur, y_new)

        # ---- the restoration phase starts where the line search failed (IPOPT: PrepareRestoPhaseStart
        # augments the filter with the current point; MinC_1NrmRestorationPhase / RestoIterateInitializer)
        ft, fp, fc = augment_filter(failed, ft, fp, fc, theta_k, phi_k)
        if bool(failed.any()):
            enter_resto(failed, w, mu, c, A, zL, zU, cur["f"])
            if watchdog:  # (the restoration phase ends the watchdog)
                S["in_wd"].copy_(S["in_wd"] & ~failed)
                S["wd_cnt"].copy_(torch.where(failed, 0, S["wd_cnt"]))
        S["w"].copy_(torch.where(mv, w_new, w))
        S["y"].copy_(torch.where(failed[:, None], S["y"], y_new))
        S["zL"].copy_(zL_new)
        S["zU"].copy_(zU_new)
        S["mu"].copy_(torch.where(act, mu, S["mu"]))
        S["iters"].copy_(S["iters"] + act_it.to(torch.int64))
        S["filt_t"].copy_(ft)
        S["filt_p"].copy_(fp)
        S["fcount"].copy_(fc)
        S["dwl"].copy_(dwl)
        for k in ("f", "grad", "g", "J"):
            S[k].copy_(torch.where(moved.view(-1, *([1] * (S[k].dim() - 1))), new[k], S[k]))
        if verbose > 1:
            verbose_line(E, mu, a_max, al, dw, dy, delta_w, cur, failed)


    def enter_resto(mask, w, mu, c, A, zL, zU, f0):
        """RestoIterateInitializer: x_R = the current point, D_R = diag(1 / max(1, |x_R|)),
        mu_R = max(mu, |c|_inf), p / n from the closed form of the barrier subproblem at fixed x
        (p - n = c, both positive), their bound multipliers mu_R / p, mu_R / n, the x-bound
        multipliers min(rho, z), least-squares constraint multipliers (<= constr_mult_init_max),
        an empty filter and a fresh quasi-Newton model."""
        mk, mw, mm = mask, mask[:, None], mask[:, None]
        c_inf = c.abs().amax(1) if m else zeros_B
        muR = torch.maximum(mu, c_inf)
        a = (muR[:, None] - RHO_R * c) / (2.0 * RHO_R)
        nn = a + torch.sqrt(a * a + muR[:, None] * c / (2.0 * RHO_R))
        pp = c + nn
        zp = muR[:, None] / pp
        zn = muR[:, None] / nn
        zLR = torch.where(hasL, torch.clamp(zL, max=RHO_R), torch.zeros_like(zL))
        zUR = torch.where(hasU, torch.clamp(zU, max=RHO_R), torch.zeros_like(zU))
        # least-squares multipliers of the restoration problem (IPOPT's estimate with M = I over
        # (w, p, n): the same p / n elimination as the Newton step, Sigma_p = Sigma_n = 1), kept when
        # |y|max <= constr_mult_init_max = 1e3
        _, yR, _ = kkt_qd(eye_w.expand(B, nw, nw), A, torch.full_like(c, 0.5), zLR - zUR, zp - zn, zeros_B, mask)
        yR = torch.where((yR.abs().amax(1) <= 1e3).unsqueeze(1), yR, torch.zeros_like(yR))
        thR0 = (c - pp + nn).abs().sum(1)
        S["resto"].copy_(S["resto"] | mk)
        S["n_resto"].copy_(S["n_resto"] + mk.to(torch.int64))
        for k, v in (("wR", w), ("p", pp), ("n", nn), ("zp", zp), ("zn", zn), ("zLR", zLR), ("zUR", zUR)):
            S[k].copy_(torch.where(mw, v, S[k]))
        S["y"].copy_(torch.where(mm, yR, S["y"]))
        S["muR"].copy_(torch.where(mk, muR, S["muR"]))
        S["ftR"].copy_(torch.where(mw, float("inf"), S["ftR"]))
        S["fpR"].copy_(torch.where(mw, float("inf"), S["fpR"]))
        S["fcR"].copy_(torch.where(mk, 0, S["fcR"]))
        S["thmaxR"].copy_(torch.where(mk, 1e4 * thR0.clamp(min=1.0), S["thmaxR"]))
        S["thminR"].copy_(torch.where(mk, 1e-4 * thR0.clamp(min=1.0), S["thminR"]))
        S["th_o0"].copy_(torch.where(mk, c.abs().sum(1), S["th_o0"]))
        S["ph_o0"].copy_(torch.where(mk, f0 + barrier(w, mu), S["ph_o0"]))
        S["dwlR"].copy_(torch.where(mk, 0.0, S["dwlR"]))
        lbfgs_reset(mk)

    def resto_step(actR):
        """One iteration of the restoration phase (IPOPT's MinC_1NrmRestorationPhase: the same
        interior-point method on  min rho sum(p + n) + eta/2 |D_R (x - x_R)|^2  s.t.  c(w) - p + n = 0,
        w within its bounds, p, n >= 0, eta = sqrt(mu_R)) for the instances in actR; then the test
        for the return to the regular iteration (RestoConvergenceCheck: the original infeasibility cut
        to kappa_resto = 0.9 of its value at the start, the point acceptable to the original filter
        and to the iterate where the phase began)."""
        w, y, mu = S["w"], S["y"], S["mu"]
        pp, nn, zp, zn, zLR, zUR, muR = S["p"], S["n"], S["zp"], S["zn"], S["zLR"], S["zUR"], S["muR"].clone()
        cur = {"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}
        A = jac_w(cur["J"])
        c = cons(cur["g"], w[:, nf:])
        DR2 = torch.where(xmask, 1.0 / torch.clamp(S["wR"].abs(), min=1.0) ** 2, torch.zeros_like(w))

        def terms(muv):
            eta = torch.sqrt(muv)
            gfw = torch.where(xmask, eta[:, None] * DR2 * (w - S["wR"]), torch.zeros_like(w))
            return eta, gfw

        # ---- the restoration problem's optimality error: converged = a point of local infeasibility
        cR = c - pp + nn
        eta, gfw = terms(muR)
        dual_w = gfw + (A.transpose(1, 2) @ y.unsqueeze(2)).squeeze(2) - zLR + zUR
        d_inf = torch.maximum(dual_w.abs().amax(1), torch.maximum((RHO_R - y - zp).abs().amax(1),
                                                                  (RHO_R + y - zn).abs().amax(1)))
        cl = torch.where(hasL, (w - torch.where(hasL, wl0, 0.0)) * zLR, torch.zeros_like(w))
        cu = torch.where(hasU, (torch.where(hasU, wu0, 0.0) - w) * zUR, torch.zeros_like(w))
        cp, cn = pp * zp, nn * zn
        nbR = nbounds + 2 * m
        zsum = zLR.abs().sum(1) + zUR.abs().sum(1) + zp.abs().sum(1) + zn.abs().sum(1)
        sd = torch.clamp((y.abs().sum(1) + zsum) / max(m + nbR, 1), min=100.0) / 100.0
        sc = torch.clamp(zsum / max(nbR, 1), min=100.0) / 100.0
        base = torch.maximum(d_inf / sd, cR.abs().amax(1))
        cmax = torch.maximum(torch.maximum(cl.amax(1), cu.amax(1)), torch.maximum(cp.amax(1), cn.amax(1)))
        errR0 = torch.maximum(base, cmax / sc)
        # converged (RestoConvergenceCheck): local infeasibility unless the original max |c| <= 1e2 tol;
        # a feasible point unacceptable to the original filter tightens the restoration tolerance to
        # 1e-2 tol once and goes on, the second time it ends the solve as a restoration failure
        tight = S["resto_tight"]
        conv = actR & (errR0 <= torch.where(tight, 1e-2 * tol, tol))
        feas = (c.abs().amax(1) if m else zeros_B) <= 1e2 * tol
        stop = conv & (~feas | tight)
        # a failed restoration phase with a backup acceptable point: IPOPT restores that point and stops
        # there (BacktrackingLineSearch: RestoreAcceptablePoint, STOP_AT_ACCEPTABLE_POINT)
        back_acc = stop & feas & S["has_acc"]
        if _DEBUG_EVENT is not None and bool(back_acc.any()):  # (diagnostics / tests)
            _DEBUG_EVENT("restore_acceptable_point", back_acc.clone())
        for k, kk in (("w", "acc_w"), ("y", "acc_y"), ("zL", "acc_zL"), ("zU", "acc_zU")):
            S[k].copy_(torch.where(back_acc[:, None], S[kk], S[k]))
        S["status"].copy_(torch.where(back_acc, STATUS_ACCEPTABLE, torch.where(stop & feas, STATUS_RESTO_FAILED,
                                      torch.where(stop, STATUS_INFEASIBLE, S["status"]))))
        S["resto_tight"].copy_(tight | (conv & feas))
        S["active"].copy_(S["active"] & ~stop)
        actR = actR & ~stop

        def errR_mu(muv):
            cm = torch.maximum(
                torch.maximum((cl - torch.where(hasL, muv[:, None], 0.0)).abs().amax(1),
                              (cu - torch.where(hasU, muv[:, None], 0.0)).abs().amax(1)),
                torch.maximum((cp - muv[:, None]).abs().amax(1), (cn - muv[:, None]).abs().amax(1)))
            return torch.maximum(base, cm / sc)

        ftR, fpR, fcR = S["ftR"], S["fpR"], S["fcR"]
        for _ in range(MU_ROUNDS):
            upd = actR & (errR_mu(muR) <= BARRIER_TOL_FACTOR * muR) & (muR > mu_min)
            muR = torch.where(upd, torch.clamp(torch.minimum(0.2 * muR, muR ** 1.5), min=mu_min), muR)
            ftR, fpR, fcR = reset_filter(upd, ftR, fpR, fcR)
        tauR = torch.clamp(1.0 - muR, min=0.99)
        eta, gfw = terms(muR)

        def phiR(wv, pv, nv):
            prox = torch.where(xmask, DR2 * (wv - S["wR"]) ** 2, torch.zeros_like(wv)).sum(1)
            return RHO_R * (pv.sum(1) + nv.sum(1)) + 0.5 * eta * prox + barrier(wv, muR) - \
                muR * (torch.log(pv).sum(1) + torch.log(nv).sum(1))

        # ---- Newton step with p, n eliminated
        if use_bfgs:
            Hc = S["Hq"]
        else:
            Hc = hessian_blk(w, y, constraints_only=True)
        dl = torch.where(hasL, w - wl0, torch.ones_like(w))
        du = torch.where(hasU, wu0 - w, torch.ones_like(w))
        Sig = torch.where(hasL, zLR / dl, torch.zeros_like(w)) + torch.where(hasU, zUR / du, torch.zeros_like(w))
        gphi = gfw - torch.where(hasL, muR[:, None] / dl, torch.zeros_like(w)) + \
            torch.where(hasU, muR[:, None] / du, torch.zeros_like(w))
        r1 = -(gphi + (A.transpose(1, 2) @ y.unsqueeze(2)).squeeze(2))
        Sp, Sn = zp / pp, zn / nn
        rp = -((RHO_R - muR[:, None] / pp) - y)
        rn = -((RHO_R - muR[:, None] / nn) + y)
        Dinv = 1.0 / (1.0 / Sp + 1.0 / Sn)
        r2 = -cR + rp / Sp - rn / Sn
        W = torch.diag_embed(Sig + torch.where(xmask, eta[:, None] * DR2, torch.zeros_like(w)))
        W[:, :nf, :nf] += Hc
        dw, dy, dWR = kkt_qd(W, A, Dinv, r1, r2, S["dwlR"], actR)
        S["dwlR"].copy_(torch.where(actR, dWR, S["dwlR"]))
        dp = (rp + dy) / Sp
        dn = (rn - dy) / Sn
        dzL = torch.where(hasL, muR[:, None] / dl - zLR - zLR / dl * dw, torch.zeros_like(w))
        dzU = torch.where(hasU, muR[:, None] / du - zUR + zUR / du * dw, torch.zeros_like(w))
        dzp = muR[:, None] / pp - zp - zp / pp * dp
        dzn = muR[:, None] / nn - zn - zn / nn * dn
        allm = torch.ones(B, m, dtype=torch.bool, device=dev)
        a_max = torch.minimum(torch.minimum(max_step(w, dw, hasL, wl0, tauR), max_step(-w, -dw, hasU, -wu0, tauR)),
                              torch.minimum(max_step(pp, dp, allm, 0.0, tauR), max_step(nn, dn, allm, 0.0, tauR)))
        a_z = torch.minimum(torch.minimum(max_step(zLR, dzL, hasL, 0.0, tauR), max_step(zUR, dzU, hasU, 0.0, tauR)),
                            torch.minimum(max_step(zp, dzp, allm, 0.0, tauR), max_step(zn, dzn, allm, 0.0, tauR)))
        gd = (gphi * dw).sum(1) + ((RHO_R - muR[:, None] / pp) * dp).sum(1) + ((RHO_R - muR[:, None] / nn) * dn).sum(1)
        thetaR = cR.abs().sum(1)
        phR_k = phiR(w, pp, nn)
        switch_ok = thetaR <= S["thminR"]
        a_min = alpha_min_of(thetaR, gd, S["thminR"])

        # ---- filter line search on the restoration problem (no second-order correction)
        st = {"searching": actR.clone(), "found": bool_B(), "f": cur["f"].clone(), "g": cur["g"].clone(),
              "w": w.clone(), "alpha": zB(), "aug": bool_B(), "p": pp.clone(), "n": nn.clone()}
        alpha = a_max.clone()
        for ls in range(max(1, max_ls)):
            if not bool(st["searching"].any()):
                break
            wt, o = trial_ls(w, dw, alpha, st["searching"], st)
            pt = pp + alpha[:, None] * dp
            nt = nn + alpha[:, None] * dn
            th_t = (cons(o["g"], wt[:, nf:]) - pt + nt).abs().sum(1)
            ph_t = phiR(wt, pt, nt)
            ok, h = acceptable(th_t, ph_t, thetaR, phR_k, gd, alpha, switch_ok, S["thmaxR"], ftR, fpR)
            take(st, st["searching"] & ok, wt, o, alpha, h, extra={"p": pt, "n": nt})
            alpha = torch.where(st["searching"], 0.5 * alpha, alpha)
            st["searching"] = st["searching"] & (alpha > a_min)
        failedR = actR & ~st["found"]
        # the restoration problem's line search failed: IPOPT's RestoRestorationPhase — w and every
        # multiplier stay, p and n take the closed-form minimisers of the barrier subproblem at the
        # current c(w) and mu_R (as at the phase's start), and that is the next iterate
        if bool(failedR.any()):
            aR = (muR[:, None] - RHO_R * c) / (2.0 * RHO_R)
            nR_ = aR + torch.sqrt(aR * aR + muR[:, None] * c / (2.0 * RHO_R))
            S["n"].copy_(torch.where(failedR[:, None], nR_, S["n"]))
            S["p"].copy_(torch.where(failedR[:, None], c + nR_, S["p"]))
        moved = actR & st["found"]
        mv = moved[:, None]
        w_new, al = st["w"], st["alpha"]
        new = evaluate(unpack(w_new))
        ftR, fpR, fcR = augment_filter(st["aug"] & moved, ftR, fpR, fcR, thetaR, phR_k)
        # accept: multipliers (alpha_y = alpha), bound multipliers with the kappa_Sigma safeguard (mu_R)
        y_new = torch.where(mv, y + al[:, None] * dy, y)

        def safeguard(zv, dz, slack, has):
            zv2 = zv + a_z[:, None] * dz
            zv2 = torch.minimum(torch.maximum(zv2, muR[:, None] / (KAPPA_SIGMA * slack)),
                                KAPPA_SIGMA * muR[:, None] / slack)
            return torch.where(mv & has, zv2, zv)

        p_new, n_new = st["p"], st["n"]
        dln = torch.where(hasL, w_new - wl0, torch.ones_like(w))
        dun = torch.where(hasU, wu0 - w_new, torch.ones_like(w))
        zLR_n = safeguard(zLR, dzL, dln, hasL)
        zUR_n = safeguard(zUR, dzU, dun, hasU)
        zp_n = safeguard(zp, dzp, p_new, allm)
        zn_n = safeguard(zn, dzn, n_new, allm)
        if use_bfgs:  # the restoration phase's own model: pairs from J^T y (its constraint curvature)
            lbfgs_update(moved, (w_new - w)[:, :nf], new, cur, y_new, with_grad=False)
        for k, v in (("p", p_new), ("n", n_new), ("zp", zp_n), ("zn", zn_n), ("zLR", zLR_n), ("zUR", zUR_n)):
            S[k].copy_(torch.where(mv, v, S[k]))
        S["w"].copy_(torch.where(mv, w_new, w))
        S["y"].copy_(y_new)
        S["muR"].copy_(torch.where(actR, muR, S["muR"]))
        S["ftR"].copy_(ftR)
        S["fpR"].copy_(fpR)
        S["fcR"].copy_(fcR)
        S["iters"].copy_(S["iters"] + actR.to(torch.int64))
        for k in ("f", "grad", "g", "J"):
            S[k].copy_(torch.where(moved.view(-1, *([1] * (S[k].dim() - 1))), new[k], S[k]))

        # ---- back to the regular iteration? (RestoConvergenceCheck / TestOrigProgress)
        c_o = cons(new["g"], w_new[:, nf:])
        th_o = c_o.abs().sum(1)
        ph_o = new["f"] + barrier(w_new, mu)
        fin = torch.isfinite(th_o) & torch.isfinite(ph_o)
        in_filter = ((th_o[:, None] <= S["filt_t"]) | (ph_o[:, None] <= S["filt_p"])).all(1)
        t0, p0 = S["th_o0"], S["ph_o0"]
        vs_start = (th_o - (1.0 - GAMMA_TH) * t0 <= 10.0 * EPS * t0.abs()) | \
            ((ph_o - p0) - (-GAMMA_PHI * t0) <= 10.0 * EPS * p0.abs())
        back = moved & fin & (th_o <= KAPPA_RESTO * S["th_o0"]) & in_filter & vs_start
        if verbose > 1:
            b = verbose_instance
            if bool(actR[b] | failedR[b]):
                print(f"   [{b}] RESTO muR={float(muR[b]):.2e} errR={float(errR0[b]):.2e} thR={float(thetaR[b]):.2e} "
                      f"a_max={float(a_max[b]):.2e} alpha={float(al[b]):.2e} th_o={float(th_o[b]):.2e} "
                      f"th_o0={float(S['th_o0'][b]):.2e} ph_o={float(ph_o[b]):.6e} ph_o0={float(S['ph_o0'][b]):.6e} "
                      f"filter={bool(in_filter[b])} start={bool(vs_start[b])} back={bool(back[b])} "
                      f"failed={bool(failedR[b])} dWR={float(dWR[b]):.1e}")
        if bool(back.any()):
            leave_resto(back, w_new, mu)

    def leave_resto(mask, w_new, mu):
        """The return to the regular iteration (MinC_1NrmRestorationPhase::PerformRestoration after
        convergence): the original bound multipliers take the primal-dual step to the new point
        (ComputeBoundMultiplierStep, dual fraction to the boundary), all of them reset to 1 when any
        exceeds bound_mult_reset_threshold = 1000; the constraint multipliers reset to 0
        (constr_mult_reset_threshold = 0); the quasi-Newton model restarts."""
        mw = mask[:, None]
        zL, zU = S["zL"], S["zU"]
        wR = S["wR"]
        tau = torch.clamp(1.0 - mu, min=0.99)
        slL0 = torch.where(hasL, wR - wl0, torch.ones_like(wR))
        slU0 = torch.where(hasU, wu0 - wR, torch.ones_like(wR))
        slL1 = torch.where(hasL, w_new - wl0, torch.ones_like(wR))
        slU1 = torch.where(hasU, wu0 - w_new, torch.ones_like(wR))
        dzL = torch.where(hasL, (zL * (slL0 - slL1) + mu[:, None]) / slL0 - zL, torch.zeros_like(zL))
        dzU = torch.where(hasU, (zU * (slU0 - slU1) + mu[:, None]) / slU0 - zU, torch.zeros_like(zU))
        a_d = torch.minimum(max_step(zL, dzL, hasL, 0.0, tau), max_step(zU, dzU, hasU, 0.0, tau))
        zLn = torch.where(hasL, zL + a_d[:, None] * dzL, zL)
        zUn = torch.where(hasU, zU + a_d[:, None] * dzU, zU)
        big = torch.maximum(zLn.amax(1), zUn.amax(1)) > BOUND_MULT_RESET
        zLn = torch.where(big[:, None] & hasL, torch.ones_like(zLn), zLn)
        zUn = torch.where(big[:, None] & hasU, torch.ones_like(zUn), zUn)
        S["zL"].copy_(torch.where(mw, zLn, zL))
        S["zU"].copy_(torch.where(mw, zUn, zU))
        S["y"].copy_(torch.where(mw, 0.0, S["y"]))
        S["resto"].copy_(S["resto"] & ~mask)
        S["acc"].copy_(torch.where(mask, 0, S["acc"]))
        lbfgs_reset(mask)

    def step():
        """One lock-step iteration: the regular iteration of the instances outside the restoration
        phase and a restoration-phase iteration of those inside it."""
        cur = {"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}
        E = errors(cur, S["w"], S["y"], S["zL"], S["zU"])
        check(E, ~S["resto"])
        actR = S["active"] & S["resto"]
        act = S["active"] & ~S["resto"]
        if bool(act.any()):
            regular_step(E, act)
        if bool(actR.any()):
            resto_step(actR)
        if fallback_viol_tol > 0:
            track_best()

    def verbose_line(E, mu, a_max, al, dw, dy, delta_w, cur, failed):
        b = verbose_instance
        print(f"   [{b}] mu={float(mu[b]):.2e} err0={float(E['err0'][b]):.2e} a_max={float(a_max[b]):.2e} "
              f"alpha={float(al[b]):.2e} dw={float(dw[b].abs().max()):.2e} dy={float(dy[b].abs().max()):.2e} "
              f"dW={float(delta_w[b]):.1e} f={float(cur['f'][b]):.6e} d_inf={float(E['d_inf'][b]):.2e} "
              f"c_inf={float(E['c_inf'][b]):.2e} resto_next={bool(failed[b])} tiny={bool(S['tiny_last'][b])}")
        if verbose > 2 and n >= 12:
            Xb = unpack(S["w"])[b]
            print("        F:", " ".join(f"({float(Xb[3+9*i]):.3g},{float(Xb[4+9*i]):.3g},{float(Xb[5+9*i]):.3g})"
                                       for i in range((n - 3) // 9)))

    # ---- drive the iterations
    it_run = 0
    while it_run < max_iter:
        if it_run % max(1, check_every) == 0 and not bool(S["active"].any()):
            break
        step()
        it_run += 1
        if verbose:
            print(f"it {it_run:4d} active {int(S['active'].sum())} resto {int((S['resto'] & S['active']).sum())}")
    # final convergence test at the last iterate (instances still in the restoration phase keep max_iter)
    check(errors({"f": S["f"], "grad": S["grad"], "g": S["g"], "J": S["J"]}, S["w"], S["y"], S["zL"], S["zU"]),
          ~S["resto"])
    fallback = bool_B()
    if fallback_viol_tol > 0:  # an unconverged instance stopped at an infeasible iterate: its best feasible one
        fallback = (S["status"] > STATUS_ACCEPTABLE) & (orig_violation(S["g"]) > fallback_viol_tol) & \
            torch.isfinite(S["best_f"])
        S["w"].copy_(torch.where(fallback[:, None], S["best_w"], S["w"]))
    # IPOPT honor_original_bounds: the final point is projected back into the unrelaxed bounds and
    # its objective / constraint values reported there
    Xf = torch.minimum(torch.maximum(unpack(S["w"]), xl), xu).contiguous()
    n_eval += 1
    fin = ev(Xf, Mass, outputs=("g", "f"))  # the unscaled callbacks
    g = fin["g"]
    viol = torch.clamp(torch.maximum(gl - g, g - gu), min=0.0).amax(1) if m else zeros_B
    res = BatchSolveResult(x=Xf, y=y_raw(S["y"]), status=S["status"],
                           iterations=S["iters"],
                           objective=fin["f"].clone(), primal_inf=viol, dual_inf=S["d_inf"], evaluations=n_eval,
                           iterations_run=it_run, graph=False)
    res.restorations = S["n_resto"]
    res.nan_jacobian = nan_jacobian
    res.fallback = fallback
    return res
