"""ctypes view of the C-ABI declared in include/cpl_mi355x.h.

Loads ``centroidalplanner_amd/libcpl_mi355x.so`` (built in-tree by ``centroidalplanner_amd.build``).
There is no fallback: if the library is missing the import of this module raises, so nothing can
silently run on a CPU path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_size_t, c_uint8, c_void_p

MAX_CONTACTS = 32
ABI_VERSION = 1

ENV_NONE = 0
ENV_GROUND = 1
ENV_SUPERQUADRIC = 2
ENV_MIXED = 3

OK = 0
ERR_INVALID_ARGUMENT = 1
ERR_OUT_OF_RANGE = 2
ERR_RUNTIME = 3
ERR_HIP = 4
ERR_UNSUPPORTED = 5

INF = 1.0e20

# cpl_eval_batch_ex output layout flags
EVAL_JAC_FOLDED = 1
EVAL_SOA = 2

LIB_NAME = "libcpl_mi355x.so"
# CPL_LIB: measurement-only override (A/B of two builds of the same ABI)
LIB_PATH = os.environ.get("CPL_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

_V3 = c_double * 3
_V3N = _V3 * MAX_CONTACTS


class ProblemDesc(ctypes.Structure):
    """Mirror of ``cpl_problem_desc`` (field order and types must match the header)."""

    _fields_ = [
        ("abi_version", c_int32),
        ("n_contacts", c_int32),
        ("env_kind", c_int32),
        ("reserved0", c_int32),
        ("map_order", c_int32 * MAX_CONTACTS),
        ("mass", c_double),
        ("gravity", c_double * 3),
        ("wrench", c_double * 6),
        ("mu", c_double),
        ("ground_z", c_double),
        ("sq_C", c_double * 3),
        ("sq_R", c_double * 3),
        ("sq_P", c_double * 3),
        ("F_thr", c_double * MAX_CONTACTS),
        ("W_com", c_double),
        ("com_ref", c_double * 3),
        ("W_p", c_double * MAX_CONTACTS),
        ("W_F", c_double * MAX_CONTACTS),
        ("p_ref", _V3N),
        ("F_ref", _V3N),
        ("com_lb", c_double * 3),
        ("com_ub", c_double * 3),
        ("F_lb", _V3N),
        ("F_ub", _V3N),
        ("p_lb", _V3N),
        ("p_ub", _V3N),
        ("n_lb", _V3N),
        ("n_ub", _V3N),
    ]


class SolveOptions(ctypes.Structure):
    """cpl_solve_options (include/cpl_mi355x.h)."""

    _fields_ = [
        ("max_iter", c_int32),
        ("hessian", c_int32),
        ("max_ls", c_int32),
        ("max_soc", c_int32),
        ("acceptable_iter", c_int32),
        ("use_graph", c_int32),
        ("compact", c_int32),
        ("ls_kernel", c_int32),
        ("tol", c_double),
        ("acceptable_tol", c_double),
        ("mu_init", c_double),
        ("fd_step", c_double),
        ("fallback_viol_tol", c_double),
        ("nlp_scaling", c_int32),
        ("jacobian_regularization", c_int32),
    ]


class DerivativeReport(ctypes.Structure):
    """cpl_derivative_report (include/cpl_mi355x.h)."""

    _fields_ = [
        ("n_checked", c_int64),
        ("n_flagged", c_int64),
        ("max_rel_error", c_double),
        ("worst_instance", c_int64),
        ("worst_row", c_int32),
        ("worst_col", c_int32),
        ("worst_exact", c_double),
        ("worst_approx", c_double),
    ]


HESSIAN_EXACT = 0
HESSIAN_LIMITED_MEMORY = 1
HESSIAN_FD = 2

# every symbol include/cpl_mi355x.h declares, with its ctypes signature
_DESC_P = POINTER(ProblemDesc)
_DP = POINTER(c_double)
_IP = POINTER(c_int32)
SIGNATURES = {
    "cpl_abi_version": (c_int32, []),
    "cpl_desc_sizeof": (c_size_t, []),
    "cpl_last_error": (c_char_p, []),
    "cpl_status_string": (c_char_p, [c_int32]),
    "cpl_desc_init": (c_int32, [_DESC_P, c_int32, c_int32, c_double]),
    "cpl_desc_set_contact_names": (c_int32, [_DESC_P, POINTER(c_char_p), c_int32]),
    "cpl_desc_set_mu": (c_int32, [_DESC_P, c_double]),
    "cpl_desc_set_superquadric": (c_int32, [_DESC_P, _DP, _DP, _DP]),
    "cpl_desc_set_bounds": (c_int32, [_DESC_P, c_int32, c_int32, _DP, _DP]),
    "cpl_dims": (c_int32, [_DESC_P, _IP, _IP, _IP]),
    "cpl_structure": (c_int32, [_DESC_P, _IP, _IP, _IP]),
    "cpl_bounds": (c_int32, [_DESC_P, _DP, _DP, _DP, _DP]),
    "cpl_eval_batch": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cpl_set_tuning": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "cpl_residual_norms": (c_int32, [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p]),
    "cpl_eval_batch_norms": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cpl_time_eval_batch": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_int32, _DP],
    ),
    "cpl_eval_batch_ex": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
         c_void_p],
    ),
    "cpl_jac_fold_info": (c_int32, [_DESC_P, _IP, _IP, _IP, _IP, _DP]),
    "cpl_time_eval_batch_ex": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_int32, c_void_p, c_int32, _DP],
    ),
    "cpl_eval_batch_host": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32],
    ),
    "cpl_derivative_test": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_double, c_double, c_void_p, POINTER(DerivativeReport),
         c_void_p],
    ),
    "cpl_kkt_workspace_doubles": (c_int64, [c_int32, c_int32]),
    "cpl_lagrangian_hessian": (c_int32, [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                         c_void_p]),
    "cpl_eval_lagrangian_grad": (
        c_int32,
        [_DESC_P, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
         c_void_p, c_void_p],
    ),
    "cpl_lagrangian_grad": (
        c_int32,
        [c_int64, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
         c_void_p, c_void_p],
    ),
    "cpl_kkt_qd_solve": (c_int32, [c_int64, c_int32, c_int32] + [c_void_p] * 12),
    "cpl_kkt_solve": (
        c_int32,
        [c_int32, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "cpl_ipm_trial_point": (
        c_int32,
        [c_int64, c_int32, c_int32, c_int32] + [c_void_p] * 11,
    ),
    "cpl_ipm_judge_take": (
        c_int32,
        [c_int64, c_int32, c_int32, c_int32, c_int32] + [c_void_p] * 27 + [c_int32, c_void_p],
    ),
    "cpl_ipm_optimality": (
        c_int32,
        [c_int64, c_int32, c_int32, c_int32, c_int32, c_double, c_double, c_int32] + [c_void_p] * 26,
    ),
    "cpl_ipm_max_step": (c_int32, [c_int64, c_int32] + [c_void_p] * 11),
    "cpl_ipm_newton_setup": (c_int32, [c_int64, c_int32, c_int32, c_int32] + [c_void_p] * 14 + [c_int32]
                             + [c_void_p] * 9),
    "cpl_ipm_fd_hessian_raw": (c_int32, [c_int64, c_int32, c_int32] + [c_void_p] * 6),
    "cpl_ipm_fd_points": (c_int32, [c_int64, c_int32, c_int32, c_double] + [c_void_p] * 6),
    "cpl_ipm_post_step": (c_int32, [c_int64, c_int32] + [c_void_p] * 23),
    "cpl_ipm_accept": (c_int32, [c_int64, c_int32, c_int32, c_int32] + [c_void_p] * 30),
    "cpl_ipm_masked_rows": (c_int32, [c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cpl_ipm_dense_a": (c_int32, [c_int64, c_int32, c_int32, c_int32, c_int32] + [c_void_p] * 6),
    "cpl_solve_options_default": (None, [POINTER(SolveOptions)]),
    "cpl_solver_create": (c_int32, [_DESC_P, c_int64, POINTER(SolveOptions), POINTER(c_void_p)]),
    "cpl_solver_destroy": (c_int32, [c_void_p]),
    "cpl_solver_solve": (c_int32, [c_void_p] + [c_void_p] * 10 + [POINTER(c_int32), POINTER(c_int64), c_void_p]),
    "cpl_solver_dims": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "cpl_solver_stats": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int64)]),
    "cpl_solver_restorations": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "cpl_solver_fallbacks": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "cpl_solver_nan_jacobian": (c_int32, [c_void_p, c_void_p, c_void_p]),
}


class CplError(RuntimeError):
    """A non-zero status from the C-ABI."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{message} (status {status})")
        self.status = status
        self.message = message


class InvalidArgument(CplError, ValueError):
    """Reference: std::invalid_argument."""


class OutOfRange(CplError, IndexError):
    """Reference: std::out_of_range."""


def _hip_runtimes_mapped():
    try:
        with open("/proc/self/maps") as fh:
            return sorted({ln.split()[-1] for ln in fh if "libamdhip64" in ln})
    except OSError:  # pragma: no cover
        return []


def _load():
    # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (DT_NEEDED
    # "libamdhip64.so", SONAME libamdhip64.so.7); this library needs "libamdhip64.so.7".  If torch
    # is importable, let it load its runtime first: our DT_NEEDED then binds to that already-loaded
    # SONAME instead of mapping /opt/rocm's copy as a second, device-less runtime.
    try:
        import torch  # noqa: F401
    except ImportError:  # C++/ctypes hosts without torch use /opt/rocm's runtime
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')"
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()

if len(_hip_runtimes_mapped()) > 1:  # pragma: no cover - would make every launch fail
    raise ImportError(f"two HIP runtimes mapped in this process: {_hip_runtimes_mapped()}")


def check(status: int) -> None:
    if status == OK:
        return
    msg = lib.cpl_last_error().decode(errors="replace")
    if status == ERR_INVALID_ARGUMENT:
        raise InvalidArgument(status, msg)
    if status == ERR_OUT_OF_RANGE:
        raise OutOfRange(status, msg)
    raise CplError(status, msg)


def dptr(a) -> ctypes.POINTER(c_double):
    return a.ctypes.data_as(POINTER(c_double))


def iptr(a) -> ctypes.POINTER(c_int32):
    return a.ctypes.data_as(POINTER(c_int32))


if lib.cpl_desc_sizeof() != ctypes.sizeof(ProblemDesc):  # pragma: no cover - layout guard
    raise ImportError("cpl_problem_desc layout mismatch between header and ctypes mirror")
