"""ctypes wrapper of the CPU restatement (oracle/cpl_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.  It is the
parity checker and the CPU baseline; the product (centroidalplanner_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CPL_ORACLE_LIB: another build of the same sources (scripts/sanitize.sh points it at the ASan/UBSan one)
LIB_PATH = os.environ.get("CPL_ORACLE_LIB") or os.path.join(HERE, "_build", "libcpl_oracle.so")


def _load(path=LIB_PATH):
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    lib = ctypes.CDLL(path)
    IP = POINTER(c_int32)
    DP = POINTER(c_double)
    lib.cplo_dims.argtypes = [c_void_p, IP, IP, IP]
    lib.cplo_dims.restype = c_int
    lib.cplo_structure.argtypes = [c_void_p, IP, IP]
    lib.cplo_structure.restype = c_int
    lib.cplo_bounds.argtypes = [c_void_p, DP, DP, DP, DP]
    lib.cplo_bounds.restype = c_int
    lib.cplo_eval_batch.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int]
    lib.cplo_eval_batch.restype = c_int
    lib.cplo_time_eval_batch.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_int, c_int]
    lib.cplo_time_eval_batch.restype = c_double
    lib.cplo_max_threads.argtypes = []
    lib.cplo_max_threads.restype = c_int
    lib.cplo_solve.argtypes = [c_void_p, c_void_p, c_double, c_int, c_double, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]
    lib.cplo_solve.restype = c_int
    lib.cplo_time_solve.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_int, c_double, c_int, c_void_p, c_void_p]
    lib.cplo_time_solve.restype = c_double
    lib.cplo_time_solve_mt.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_int, c_double, c_int, c_int, c_void_p,
                                       c_void_p]
    lib.cplo_time_solve_mt.restype = c_double
    lib.cplo_set_fallback_viol_tol.argtypes = [c_double]
    lib.cplo_set_fallback_viol_tol.restype = None
    lib.cplo_set_nlp_scaling.argtypes = [c_int]
    lib.cplo_set_nlp_scaling.restype = None
    lib.cplo_set_watchdog.argtypes = [c_int]
    lib.cplo_set_watchdog.restype = None
    lib.cplo_set_acceptable_tol.argtypes = [c_double]
    lib.cplo_set_watchdog_params.argtypes = [c_int, c_int]
    lib.cplo_set_watchdog_params.restype = None
    lib.cplo_set_acceptable_tol.restype = None
    lib.cplo_watchdog_events.argtypes = [ctypes.POINTER(ctypes.c_long)]
    lib.cplo_watchdog_events.restype = None
    lib.cplo_resto_fail_events.argtypes = [ctypes.POINTER(ctypes.c_long)]
    lib.cplo_resto_fail_events.restype = None
    lib.cplo_set_jac_reg.argtypes = [c_int]
    lib.cplo_set_jac_reg.restype = None
    return lib


lib = _load()
_variants = {}


def variant_lib(name):
    """The oracle built with a variant switch: "novec" = Eigen's non-vectorised 3-vector reduction
    order a0 b0 + (a1 b1 + a2 b2) (cpl_oracle.c CPLO_EIGEN_REDUX_NOVEC) instead of SSE2's."""
    if name not in _variants:
        _variants[name] = _load(os.path.join(HERE, "_build", f"libcpl_oracle_{name}.so"))
    return _variants[name]


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def dims(desc):
    n, m, nnz = c_int32(), c_int32(), c_int32()
    st = lib.cplo_dims(ctypes.byref(desc), ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz))
    if st:
        raise ValueError(f"oracle dims failed: {st}")
    return n.value, m.value, nnz.value


def structure(desc):
    _, _, nnz = dims(desc)
    iRow = np.zeros(nnz, dtype=np.int32)
    jCol = np.zeros(nnz, dtype=np.int32)
    st = lib.cplo_structure(ctypes.byref(desc), iRow.ctypes.data_as(POINTER(c_int32)),
                            jCol.ctypes.data_as(POINTER(c_int32)))
    if st:
        raise ValueError(f"oracle structure failed: {st}")
    return iRow, jCol


def bounds(desc):
    n, m, _ = dims(desc)
    xl, xu, gl, gu = np.zeros(n), np.zeros(n), np.zeros(m), np.zeros(m)
    DP = POINTER(c_double)
    st = lib.cplo_bounds(ctypes.byref(desc), xl.ctypes.data_as(DP), xu.ctypes.data_as(DP), gl.ctypes.data_as(DP),
                         gu.ctypes.data_as(DP))
    if st:
        raise ValueError(f"oracle bounds failed: {st}")
    return xl, xu, gl, gu


def eval_batch(desc, x, mass=None, env_tag=None, outputs=("g", "jac", "f", "grad"), nthreads=None, variant=None):
    """x: float64 [B, n] host array.  Returns dict of host arrays.  variant: see variant_lib."""
    L = lib if variant is None else variant_lib(variant)
    n, m, nnz = dims(desc)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, n)
    B = x.shape[0]
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    env_tag = None if env_tag is None else np.ascontiguousarray(env_tag, dtype=np.uint8)
    shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n)}
    out = {k: np.zeros(shapes[k]) for k in outputs}
    if nthreads is None:
        nthreads = L.cplo_max_threads()
    st = L.cplo_eval_batch(ctypes.byref(desc), B, _p(x), _p(mass), _p(env_tag), _p(out.get("g")),
                             _p(out.get("jac")), _p(out.get("f")), _p(out.get("grad")), int(nthreads))
    if st:
        raise ValueError(f"oracle eval failed: {st}")
    return out


def time_eval_batch(desc, x, mass=None, env_tag=None, outputs=("g", "jac"), nthreads=1, reps=1):
    """Seconds per batch evaluation (wall clock inside the C library)."""
    n, m, nnz = dims(desc)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, n)
    B = x.shape[0]
    shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n)}
    out = {k: np.zeros(shapes[k]) for k in outputs}
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    env_tag = None if env_tag is None else np.ascontiguousarray(env_tag, dtype=np.uint8)
    t = lib.cplo_time_eval_batch(ctypes.byref(desc), B, _p(x), _p(mass), _p(env_tag), _p(out.get("g")),
                                 _p(out.get("jac")), _p(out.get("f")), _p(out.get("grad")), int(nthreads), int(reps))
    if t < 0:
        raise ValueError("oracle timing failed")
    return t


STATUS_NAMES = ("optimal", "acceptable", "max_iter", "infeasible", "resto_failed")


def solve(desc, x0, mass=None, max_iter=3000, tol=1e-8, hessian="limited-memory"):
    """One solve on this thread by the compiled restatement of the solve loop (cpl_solve_host.c:
    IPOPT's iteration with IFOPT's limited-memory Hessian, or hessian="exact": the analytic one;
    IPOPT itself absent).  Returns a dict:
    x [n], status (0 optimal .. 4, STATUS_NAMES), iterations, objective, restorations, evaluations."""
    n, _, _ = dims(desc)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(n)
    x = np.zeros(n)
    st, it, rs = c_int32(), c_int32(), c_int32()
    obj, ev = c_double(), c_int64()
    r = lib.cplo_solve(ctypes.byref(desc), _p(x0), float(desc.mass if mass is None else mass), int(max_iter),
                       float(tol), int(hessian == "exact"), _p(x), ctypes.byref(st), ctypes.byref(it), ctypes.byref(obj), ctypes.byref(rs),
                       ctypes.byref(ev))
    if r:
        raise ValueError(f"oracle solve failed: {r}")
    return {"x": x, "status": st.value, "iterations": it.value, "objective": obj.value, "restorations": rs.value,
            "evaluations": ev.value}


def time_solve(desc, x0, mass=None, max_iter=3000, tol=1e-8, hessian="limited-memory"):
    """Wall-clock seconds of sequential single-thread solves of x0 [count, n] (the CPU baseline of the
    solve legs); returns (seconds, status [count], iterations [count])."""
    n, _, _ = dims(desc)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, n)
    cnt = x0.shape[0]
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    st = np.zeros(cnt, dtype=np.int32)
    it = np.zeros(cnt, dtype=np.int32)
    t = lib.cplo_time_solve(ctypes.byref(desc), cnt, _p(x0), _p(mass), int(max_iter), float(tol), int(hessian == "exact"),
                            _p(st), _p(it))
    if t < 0:
        raise ValueError("oracle solve timing failed")
    return t, st, it


def time_solve_mt(desc, x0, mass=None, max_iter=3000, tol=1e-8, hessian="limited-memory", threads=0):
    """time_solve over `threads` OpenMP threads (0: all of OMP_NUM_THREADS / the affinity mask), the
    instances split dynamically: the all-core CPU baseline of the solve legs.  Every instance takes the
    iterates of its single-thread solve (the solver state is per thread)."""
    n, _, _ = dims(desc)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, n)
    cnt = x0.shape[0]
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    st = np.zeros(cnt, dtype=np.int32)
    it = np.zeros(cnt, dtype=np.int32)
    t = lib.cplo_time_solve_mt(ctypes.byref(desc), cnt, _p(x0), _p(mass), int(max_iter), float(tol),
                               int(hessian == "exact"), int(threads), _p(st), _p(it))
    if t < 0:
        raise ValueError("oracle solve timing failed")
    return t, st, it


def set_fallback_viol_tol(v):
    """Opt in to the best-feasible-iterate fallback (not IPOPT) in the compiled restatement: v > 0;
    0 (the default, like the engine's) returns the last iterate as IPOPT does."""
    lib.cplo_set_fallback_viol_tol(float(v))


def set_nlp_scaling(method):
    """nlp_scaling_method of the compiled restatement: "gradient-based" (IPOPT's default, the
    reference's; the default here too) or "none" (process-wide)."""
    lib.cplo_set_nlp_scaling(1 if method == "gradient-based" else 0)


def set_jac_reg(on):
    """IPOPT's regularisation of a rank-deficient Jacobian ([[W, A^T], [A, -delta_c I]], delta_c = 1e-8 mu^0.25)
    in the compiled restatement (opt-in, process-wide): the measurement of what the engine's treatment (delta_c
    on R's near-zero pivots) costs TestBasic's degenerate starts."""
    lib.cplo_set_jac_reg(1 if on else 0)


def set_watchdog(on):
    """IPOPT's watchdog in the compiled restatement (opt-in, process-wide; the engine has none): the
    measurement of its effect (scripts/watchdog_effect.py)."""
    lib.cplo_set_watchdog(1 if on else 0)


def set_watchdog_params(trigger=10, trial_max=3):
    """The watchdog's watchdog_shortened_iter_trigger / watchdog_trial_iter_max (IPOPT: 10 / 3;
    process-wide; the tests lower the trigger to compare the restatements where it starts)."""
    lib.cplo_set_watchdog_params(int(trigger), int(trial_max))


def watchdog_events():
    """(starts, successes, restorations of the kept iterate) of the watchdog on this thread since the
    last call (single-thread solves)."""
    out = (ctypes.c_long * 3)()
    lib.cplo_watchdog_events(out)
    return tuple(int(v) for v in out)


def set_acceptable_tol(v):
    """IPOPT's acceptable_tol in the compiled restatement (process-wide; default 1e-6)."""
    lib.cplo_set_acceptable_tol(float(v))


def resto_fail_events():
    """(failed restoration phases ending at a feasible point, those of them that restored the backup
    acceptable point) on this thread since the last call (single-thread solves)."""
    out = (ctypes.c_long * 2)()
    lib.cplo_resto_fail_events(out)
    return tuple(int(v) for v in out)


def max_threads():
    return lib.cplo_max_threads()


def lagrangian_hessian(desc, X, Y, free_idx=None):
    """Exact Hessian of f + y^T g over the variables `free_idx` (default: all), [B, nf, nf] — the
    checker of cpl_lagrangian_hessian (csrc/cpl_kernels.hip hessian_entry) and the CPU solve loop's
    Hessian: per entry the same operations in the same order, so the GPU kernel is bitwise equal.
    Ground / no-environment problems (their environment and normal rows are linear).
      cost:   W_com, W_F,i, W_p,i on the diagonal (src/MinimizeCentroidalVariables.cpp:124-148);
      torque: d2/dp_a dF_b = E_ab, d2/dc_a dF_b = -E_ab, E_ab = sum_k y_{3+k} eps_kab
              (src/Constraints/CentroidalStatics.cpp:37-61);
      cones:  -F.n and |t| - mu F.n, t = F - (F.n) n (src/Constraints/FrictionCone.cpp:30-45); the |t|
              terms count as 0 where |t| = 0 (the reference's Jacobian is 0/0 there).
    X [B, n], Y [B, m] float64 host arrays."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    N = int(desc.n_contacts)
    n = 3 + 9 * N
    B = X.shape[0]
    crow = 6 if desc.env_kind in (1, 2, 3) else 2
    pos = np.zeros(N, dtype=np.int64)
    for k in range(N):
        pos[desc.map_order[k]] = k
    H = np.zeros((B, n, n))
    # cost diagonal: h = 0.0 + W
    for a in range(3):
        H[:, a, a] = 0.0 + desc.W_com
    for i in range(N):
        for a in range(3):
            H[:, 3 + 9 * i + a, 3 + 9 * i + a] = 0.0 + desc.W_F[i]
            H[:, 6 + 9 * i + a, 6 + 9 * i + a] = 0.0 + desc.W_p[i]
            H[:, 9 + 9 * i + a, 9 + 9 * i + a] = 0.0 + 0.0

    def E(a, c):
        if a == c:
            return np.zeros(B)
        k = 3 - a - c
        sgn = 1.0 if (a + 1) % 3 == c else -1.0
        return sgn * Y[:, 3 + k]

    for i in range(N):
        for a in range(3):
            for b in range(3):
                Fb, pa, ca = 3 + 9 * i + b, 6 + 9 * i + a, a
                H[:, pa, Fb] = 0.0 + E(a, b)       # d2/dp_a dF_b
                H[:, Fb, pa] = 0.0 + E(a, b)       # d2/dF_b dp_a (E(av, au) with v = p_a)
                H[:, ca, Fb] = 0.0 - E(a, b)       # d2/dc_a dF_b
                H[:, Fb, ca] = 0.0 - E(a, b)
    mu = desc.mu
    with np.errstate(all="ignore"):
        for i in range(N):
            q = X[:, 3 + 9 * i: 12 + 9 * i]
            F = [q[:, 0], q[:, 1], q[:, 2]]
            nn = [q[:, 6], q[:, 7], q[:, 8]]
            r0 = 6 + crow * int(pos[i]) + (crow - 2)
            y0, y1 = Y[:, r0], Y[:, r0 + 1]
            sdot = (F[0] * nn[0] + F[1] * nn[1]) + F[2] * nn[2]
            t = [F[j] - sdot * nn[j] for j in range(3)]
            rr = np.sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2])
            ok = (rr > 0.0) & (rr < np.inf) & (y1 != 0.0)
            u = [t[j] / rr for j in range(3)]

            def col(kind, a):
                if kind == 1:
                    return [(1.0 if j == a else 0.0) - nn[j] * nn[a] for j in range(3)]
                return [-(nn[j] * F[a] + (sdot if j == a else 0.0)) for j in range(3)]

            for u6 in range(6):
                for v6 in range(6):
                    ku, au = (1, u6) if u6 < 3 else (3, u6 - 3)
                    kv, av = (1, v6) if v6 < 3 else (3, v6 - 3)
                    uu = 3 + 9 * i + (u6 if u6 < 3 else 3 + u6)
                    vv = 3 + 9 * i + (v6 if v6 < 3 else 3 + v6)
                    h = H[:, uu, vv].copy()
                    fn = (ku == 1 and kv == 3) or (ku == 3 and kv == 1)
                    aF = au if ku == 1 else av
                    an = au if ku == 3 else av
                    if fn and aF == an:
                        h = h - (y0 + mu * y1)
                    cu, cv = col(ku, au), col(kv, av)
                    jj = (cu[0] * cv[0] + cu[1] * cv[1]) + cu[2] * cv[2]
                    pu = (u[0] * cu[0] + u[1] * cu[1]) + u[2] * cu[2]
                    pv = (u[0] * cv[0] + u[1] * cv[1]) + u[2] * cv[2]
                    if fn:
                        un = (u[0] * nn[0] + u[1] * nn[1]) + u[2] * nn[2]
                        second = -((un if aF == an else 0.0) + nn[aF] * u[an])
                    elif ku == 3 and kv == 3:
                        second = -(F[au] * u[av] + F[av] * u[au])
                    else:
                        second = 0.0
                    H[:, uu, vv] = np.where(ok, h + y1 * ((jj - pu * pv) / rr + second), h)
    if free_idx is not None:
        fi = np.asarray(free_idx, dtype=np.int64)
        H = H[:, fi][:, :, fi]
    return H
