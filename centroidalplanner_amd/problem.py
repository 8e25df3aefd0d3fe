"""Host-side mirror of CentroidalPlanner's problem API over the C-ABI.

Names, argument meaning and error behaviour follow the reference:
  cpl::env::EnvironmentClass / Ground / Superquadric  include/CentroidalPlanner/Environment/*.h
  cpl::solver::CplProblem                              include/CentroidalPlanner/Ifopt/CplProblem.h
plus the IPOPT TNLP hooks IFOPT's IpoptAdapter exposes [IFOPT-ext] (get_nlp_info,
get_bounds_info, get_starting_point, eval_f, eval_grad_f, eval_g, eval_jac_g), which here run on
the GPU through ``cpl_eval_batch``.  ``eval_batch`` is the batched hot path: many instances of
one problem template in a single launch, inputs and outputs resident in device memory.

PyTorch is only used for device memory and streams.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import _abi
from ._abi import (ENV_GROUND, ENV_MIXED, ENV_NONE, ENV_SUPERQUADRIC, InvalidArgument, OutOfRange, ProblemDesc,
                   check, dptr, iptr, lib)


def _v3(v) -> np.ndarray:
    a = np.asarray(v, dtype=np.float64).reshape(-1)
    if a.shape != (3,):
        raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "expected a 3-vector")
    return a


# --------------------------------------------------------------------------------------------
# Environments  (include/CentroidalPlanner/Environment/Environment.h:13-48)
# --------------------------------------------------------------------------------------------
class EnvironmentClass:
    kind = ENV_NONE

    def __init__(self):
        self._mu = 1.0  # Environment.h:46

    def SetMu(self, mu: float) -> None:  # Environment.h:19-26
        if mu <= 0.0:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid friction coefficient")
        self._mu = float(mu)

    def GetMu(self) -> float:
        return self._mu


class Ground(EnvironmentClass):
    """Flat ground z = ground_z (src/Ground.cpp)."""

    kind = ENV_GROUND

    def __init__(self):
        super().__init__()
        self._ground_z = 0.0  # src/Ground.cpp:7

    def SetGroundZ(self, ground_z: float) -> None:
        self._ground_z = float(ground_z)

    def GetGroundZ(self) -> float:
        return self._ground_z


class Superquadric(EnvironmentClass):
    """Superquadric sum_k ((p_k-C_k)/R_k)^P_k = 1 (src/Superquadric.cpp)."""

    kind = ENV_SUPERQUADRIC

    def __init__(self):
        super().__init__()
        self._C = np.array([0.0, 0.0, 10.0])  # src/Superquadric.cpp:7-9
        self._R = np.array([10.0, 10.0, 10.0])
        self._P = np.array([10.0, 10.0, 10.0])

    def SetParameters(self, C, R, P) -> None:  # src/Superquadric.cpp:12-29
        C, R, P = _v3(C), _v3(R), _v3(P)
        if (R <= 0.0).any():
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid superquadric axial radii")
        if (P < 2.0).any():
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid superquadric axial curvatures: must be >= 2")
        self._C, self._R, self._P = C.copy(), R.copy(), P.copy()

    def GetParameters(self):
        return self._C.copy(), self._R.copy(), self._P.copy()


class MixedEnvironment(EnvironmentClass):
    """A batch whose instances are each on a Ground or on a Superquadric (per-instance tag).

    Not a reference class: the reference has one environment per problem
    (include/CentroidalPlanner/Ifopt/CplProblem.h:105).  The batch mixes environments per instance.
    """

    kind = ENV_MIXED

    def __init__(self, ground: Ground, superquadric: Superquadric):
        super().__init__()
        self.ground = ground
        self.superquadric = superquadric
        self._mu = ground.GetMu()


# --------------------------------------------------------------------------------------------
# CplProblem  (src/CplProblem.cpp)
# --------------------------------------------------------------------------------------------
class CplProblem:
    """One CentroidalPlanner problem template; evaluates single instances (TNLP hooks) or batches.

    ``env=None`` is the CoMPlanner path (FrictionCone only, mu kept by a private Ground,
    src/CplProblem.cpp:14,63-71).
    """

    def __init__(self, contact_names: Sequence[str], robot_mass: float, env: Optional[EnvironmentClass]):
        names = [str(c) for c in contact_names]
        if len(names) < 1 or len(names) > _abi.MAX_CONTACTS:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "number of contacts out of range")
        self._contact_names = names
        self._env = env
        self._ground_fake = Ground()
        self._desc = ProblemDesc()
        kind = env.kind if env is not None else ENV_NONE
        check(lib.cpl_desc_init(ctypes.byref(self._desc), len(names), kind, float(robot_mass)))
        arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        check(lib.cpl_desc_set_contact_names(ctypes.byref(self._desc), arr, len(names)))
        self._index = {n: i for i, n in enumerate(names)}
        self._x = np.zeros(self.n)  # Variable3D init 0 (src/Variable3D.cpp:8-10)

    # ---- layout --------------------------------------------------------------------------
    @property
    def contact_names(self) -> List[str]:
        return list(self._contact_names)

    @property
    def map_order(self) -> List[int]:
        return [self._desc.map_order[k] for k in range(len(self._contact_names))]

    def _dims(self):
        n, m, nnz = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.cpl_dims(ctypes.byref(self._desc), ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz)))
        return n.value, m.value, nnz.value

    @property
    def n(self) -> int:
        return self._dims()[0]

    @property
    def m(self) -> int:
        return self._dims()[1]

    @property
    def nnz(self) -> int:
        return self._dims()[2]

    def _i(self, contact_name: str) -> int:
        try:
            return self._index[contact_name]
        except KeyError:  # std::map::at
            raise OutOfRange(_abi.ERR_OUT_OF_RANGE, f"map::at: no contact '{contact_name}'") from None

    def desc(self) -> ProblemDesc:
        """The problem template with the environment's current state folded in."""
        d = self._desc
        env = self._env
        if env is None:
            d.mu = self._ground_fake.GetMu()
        else:
            d.mu = env.GetMu()
            g = env.ground if isinstance(env, MixedEnvironment) else env
            s = env.superquadric if isinstance(env, MixedEnvironment) else env
            if isinstance(g, Ground):
                d.ground_z = g.GetGroundZ()
            if isinstance(s, Superquadric):
                C, R, P = s.GetParameters()
                for j in range(3):
                    d.sq_C[j], d.sq_R[j], d.sq_P[j] = C[j], R[j], P[j]
        return d

    # ---- reference setters / getters (src/CplProblem.cpp:109-316) -----------------------------
    def _set_bounds(self, var: int, contact: int, lb, ub) -> None:
        lb, ub = _v3(lb), _v3(ub)
        check(lib.cpl_desc_set_bounds(ctypes.byref(self._desc), var, contact, dptr(lb), dptr(ub)))

    def _get_bounds(self, lo, hi):
        return np.array(lo[:]), np.array(hi[:])

    def SetForceBounds(self, contact_name, force_lb, force_ub):
        self._set_bounds(1, self._i(contact_name), force_lb, force_ub)

    def GetForceBounds(self, contact_name):
        i = self._i(contact_name)
        return self._get_bounds(self._desc.F_lb[i], self._desc.F_ub[i])

    def SetPosBounds(self, contact_name, pos_lb, pos_ub):
        self._set_bounds(2, self._i(contact_name), pos_lb, pos_ub)

    def GetPosBounds(self, contact_name):
        i = self._i(contact_name)
        return self._get_bounds(self._desc.p_lb[i], self._desc.p_ub[i])

    def SetNormalBounds(self, contact_name, normal_lb, normal_ub):
        self._set_bounds(3, self._i(contact_name), normal_lb, normal_ub)

    def GetNormalBounds(self, contact_name):
        i = self._i(contact_name)
        return self._get_bounds(self._desc.n_lb[i], self._desc.n_ub[i])

    def SetCoMBounds(self, com_lb, com_ub):
        self._set_bounds(0, 0, com_lb, com_ub)

    def SetPosRef(self, contact_name, pos_ref):
        i, v = self._i(contact_name), _v3(pos_ref)
        for j in range(3):
            self._desc.p_ref[i][j] = v[j]

    def GetPosRef(self, contact_name):
        return np.array(self._desc.p_ref[self._i(contact_name)][:])

    def SetForceRef(self, contact_name, force_ref):
        i, v = self._i(contact_name), _v3(force_ref)
        for j in range(3):
            self._desc.F_ref[i][j] = v[j]

    def GetForceRef(self, contact_name):
        return np.array(self._desc.F_ref[self._i(contact_name)][:])

    def SetCoMRef(self, com_ref):
        v = _v3(com_ref)
        for j in range(3):
            self._desc.com_ref[j] = v[j]

    def GetCoMRef(self):
        return np.array(self._desc.com_ref[:])

    def SetCoMWeight(self, W_CoM):
        self._desc.W_com = float(W_CoM)

    def GetCoMWeight(self):
        return self._desc.W_com

    def SetPosWeight(self, W_p):
        for i in range(len(self._contact_names)):
            self._desc.W_p[i] = float(W_p)

    def SetContactPosWeight(self, contact_name, W_p):
        self._desc.W_p[self._i(contact_name)] = float(W_p)

    def GetContactPosWeight(self, contact_name):
        return self._desc.W_p[self._i(contact_name)]

    def SetForceWeight(self, W_F):
        for i in range(len(self._contact_names)):
            self._desc.W_F[i] = float(W_F)

    def SetContactForceWeight(self, contact_name, W_F):
        self._desc.W_F[self._i(contact_name)] = float(W_F)

    def GetContactForceWeight(self, contact_name):
        return self._desc.W_F[self._i(contact_name)]

    def SetManipulationWrench(self, wrench_manip):
        w = np.asarray(wrench_manip, dtype=np.float64).reshape(-1)
        if w.shape != (6,):
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "manipulation wrench must have 6 entries")
        for j in range(6):
            self._desc.wrench[j] = w[j]

    def GetManipulationWrench(self):
        return np.array(self._desc.wrench[:])

    def SetMass(self, m):
        self._desc.mass = float(m)

    def SetMu(self, mu):  # src/CplProblem.cpp:275-287
        (self._env if self._env is not None else self._ground_fake).SetMu(mu)

    def GetMu(self):
        return (self._env if self._env is not None else self._ground_fake).GetMu()

    def SetForceThreshold(self, contact_name, F_thr):
        self._desc.F_thr[self._i(contact_name)] = float(F_thr)

    def GetForceThreshold(self, contact_name):
        return self._desc.F_thr[self._i(contact_name)]

    # ---- IPOPT TNLP hooks [IFOPT-ext IpoptAdapter] -------------------------------------------
    def get_nlp_info(self):
        return self._dims()

    def get_structure(self):
        """eval_jac_g(values == NULL): (iRow, jCol) in RowMajor CSR order."""
        _, _, nnz = self._dims()
        iRow = np.zeros(nnz, dtype=np.int32)
        jCol = np.zeros(nnz, dtype=np.int32)
        check(lib.cpl_structure(ctypes.byref(self.desc()), iptr(iRow), iptr(jCol), None))
        return iRow, jCol

    def get_row_ptr(self):
        m = self.m
        rp = np.zeros(m + 1, dtype=np.int32)
        check(lib.cpl_structure(ctypes.byref(self.desc()), None, None, iptr(rp)))
        return rp

    def jac_fold_info(self):
        """The values-only Jacobian layout (cpl_jac_fold_info): (var_k, const_k, const_val) — the CSR
        positions of the folded values, and the positions / values of the skipped constants."""
        nf, nc = ctypes.c_int32(), ctypes.c_int32()
        check(lib.cpl_jac_fold_info(ctypes.byref(self.desc()), ctypes.byref(nf), None, ctypes.byref(nc), None, None))
        var_k = np.zeros(nf.value, dtype=np.int32)
        const_k = np.zeros(nc.value, dtype=np.int32)
        const_val = np.zeros(nc.value)
        check(lib.cpl_jac_fold_info(ctypes.byref(self.desc()), ctypes.byref(nf), iptr(var_k), ctypes.byref(nc),
                                    iptr(const_k), dptr(const_val)))
        return var_k, const_k, const_val

    def get_bounds_info(self):
        n, m, _ = self._dims()
        xl, xu, gl, gu = np.zeros(n), np.zeros(n), np.zeros(m), np.zeros(m)
        check(lib.cpl_bounds(ctypes.byref(self.desc()), dptr(xl), dptr(xu), dptr(gl), dptr(gu)))
        return xl, xu, gl, gu

    def get_starting_point(self):
        return self._x.copy()

    def SetVariables(self, x):
        self._x = np.asarray(x, dtype=np.float64).reshape(self.n).copy()

    def eval_batch_host(self, x, mass=None, env_tag=None, outputs: Iterable[str] = ("g", "jac"),
                        jac_folded: bool = False):
        """cpl_eval_batch_host: numpy arrays in and out, evaluated by the GPU kernel (staged through
        the library's device workspace; synchronous).  x: [B, n]; mass: [B] or None; env_tag: uint8
        [B] (mixed only); outputs: subset of {"g", "jac", "f", "grad", "norms"}."""
        n, m, nnz = self._dims()
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1, n))
        B = x.shape[0]
        outputs = tuple(outputs)
        if "norms" in outputs and "g" not in outputs:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "'norms' needs the 'g' output")
        if jac_folded:
            nf = ctypes.c_int32()
            check(lib.cpl_jac_fold_info(ctypes.byref(self.desc()), ctypes.byref(nf), None, None, None, None))
            nnz = nf.value
        shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n), "norms": (2,)}
        res = {}
        for k in outputs:
            if k not in shapes:
                raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"unknown output '{k}'")
            res[k] = np.empty(shapes[k])
        if mass is not None:
            mass = np.ascontiguousarray(np.asarray(mass, dtype=np.float64).reshape(B))
        if env_tag is not None:
            env_tag = np.ascontiguousarray(np.asarray(env_tag, dtype=np.uint8).reshape(B))

        def p(a):
            return ctypes.c_void_p(a.ctypes.data) if a is not None else None

        flags = _abi.EVAL_JAC_FOLDED if jac_folded else 0
        check(lib.cpl_eval_batch_host(ctypes.byref(self.desc()), B, p(x), p(mass), p(env_tag), p(res.get("g")),
                                      p(res.get("jac")), p(res.get("f")), p(res.get("grad")), p(res.get("norms")),
                                      flags))
        return res

    def derivative_test(self, x, mass=None, env_tag=None, perturbation: float = 1e-8, tol: float = 1e-4,
                        per_instance: bool = False, stream=None):
        """IPOPT's first-order derivative checker over a batch (cpl_derivative_test; the reference runs
        it on every solve, src/CentroidalPlanner.cpp:26).  x: float64 CUDA tensor [B, n].  Returns a
        dict with n_checked, n_flagged, max_rel_error, worst_instance / row (-1 = objective gradient)
        / col / exact / approx, and ``flagged`` (int32 tensor [B]) when per_instance."""
        import torch

        n, _, _ = self._dims()
        if x.dtype != torch.float64 or not x.is_cuda or x.dim() != 2 or x.shape[1] != n or not x.is_contiguous():
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"x must be a contiguous float64 CUDA tensor [B, {n}]")
        B = x.shape[0]
        flagged = torch.zeros(B, dtype=torch.int32, device=x.device) if per_instance else None
        rep = _abi.DerivativeReport()
        s = stream if stream is not None else torch.cuda.current_stream(x.device)

        def p(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        check(lib.cpl_derivative_test(ctypes.byref(self.desc()), B, p(x), p(mass), p(env_tag), float(perturbation),
                                      float(tol), p(flagged), ctypes.byref(rep), ctypes.c_void_p(s.cuda_stream)))
        out = {k: getattr(rep, k) for k, _ in _abi.DerivativeReport._fields_}
        if per_instance:
            out["flagged"] = flagged
        return out

    def _eval_one(self, x, want):
        # the single-instance IFOPT-style callback path: host arrays through cpl_eval_batch_host
        out = self.eval_batch_host(np.asarray(x, dtype=np.float64).reshape(1, -1), outputs=want)
        return {k: v[0] for k, v in out.items()}

    def eval_f(self, x) -> float:
        return float(self._eval_one(x, ("f",))["f"])

    def eval_grad_f(self, x) -> np.ndarray:
        return self._eval_one(x, ("grad",))["grad"]

    def eval_g(self, x) -> np.ndarray:
        return self._eval_one(x, ("g",))["g"]

    def eval_jac_g(self, x) -> np.ndarray:
        return self._eval_one(x, ("jac",))["jac"]

    def GetSolution(self) -> Dict:
        """Solution struct (include/CentroidalPlanner/Ifopt/Types.h:15-21): contacts in map order."""
        x = self._x
        sol = {"com": x[0:3].copy(), "contact_values_map": {}}
        for name in sorted(self._contact_names, key=lambda s: s.encode()):
            i = self._index[name]
            sol["contact_values_map"][name] = {
                "force": x[3 + 9 * i: 6 + 9 * i].copy(),
                "position": x[6 + 9 * i: 9 + 9 * i].copy(),
                "normal": x[9 + 9 * i: 12 + 9 * i].copy(),
            }
        return sol

    # ---- the batched hot path ---------------------------------------------------------------
    def eval_batch(self, x, mass=None, env_tag=None, outputs: Iterable[str] = ("g", "jac"), out=None,
                   stream=None, jac_folded: bool = False, soa: bool = False):
        """Evaluate B instances on the GPU in one launch.

        x: torch.float64 CUDA tensor [B, n] (contiguous).  mass: [B] or None.  env_tag: uint8 [B]
        (mixed environment only).  outputs: subset of {"g", "jac", "f", "grad", "norms"}; "norms"
        (with "g") fuses the per-batch residual norms [max violation, sum of squared violations]
        into the same launch (cpl_eval_batch_norms).  out: optional
        dict of preallocated output tensors.  Returns the dict of output tensors; asynchronous on
        ``stream`` (default: torch's current stream).
        jac_folded: values-only Jacobian records (structural constants skipped, see jac_fold_info);
        soa: entry-major outputs g [m, B], jac [nnz, B], grad [n, B] (cpl_eval_batch_ex).
        """
        import torch

        n, m, nnz = self._dims()
        outputs = tuple(outputs)
        want_norms = "norms" in outputs
        if want_norms and "g" not in outputs:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "'norms' needs the 'g' output")
        outputs = tuple(k for k in outputs if k != "norms")
        if x.dtype != torch.float64 or not x.is_cuda or x.dim() != 2 or x.shape[1] != n or not x.is_contiguous():
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"x must be a contiguous float64 CUDA tensor [B, {n}]")
        B = x.shape[0]
        flags = (_abi.EVAL_JAC_FOLDED if jac_folded else 0) | (_abi.EVAL_SOA if soa else 0)
        if jac_folded:
            nf = ctypes.c_int32()
            check(lib.cpl_jac_fold_info(ctypes.byref(self.desc()), ctypes.byref(nf), None, None, None, None))
            nnz = nf.value
        shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n)}
        if soa:
            shapes = {k: (v[1], v[0]) if len(v) == 2 else v for k, v in shapes.items()}
        res = {}
        for k in outputs:
            if k not in shapes:
                raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"unknown output '{k}'")
            t = out.get(k) if out else None
            if t is None:
                t = torch.empty(shapes[k], dtype=torch.float64, device=x.device)
            elif (tuple(t.shape) != shapes[k] or t.dtype != torch.float64 or not t.is_contiguous()
                  or t.device != x.device):
                raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT,
                                      f"output '{k}' must be a contiguous float64 tensor {shapes[k]} on {x.device}")
            res[k] = t
        if mass is not None and (mass.dtype != torch.float64 or tuple(mass.shape) != (B,) or mass.device != x.device
                                 or not mass.is_contiguous()):
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"mass must be a contiguous float64 tensor [B] on {x.device}")
        if env_tag is not None and (env_tag.dtype != torch.uint8 or tuple(env_tag.shape) != (B,)
                                    or env_tag.device != x.device or not env_tag.is_contiguous()):
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"env_tag must be a contiguous uint8 tensor [B] on {x.device}")
        s = stream if stream is not None else torch.cuda.current_stream(x.device)

        def p(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        if want_norms:  # fused residual norms of g: one launch, no second pass over g
            t = out.get("norms") if out else None
            if t is None:
                t = torch.empty(2, dtype=torch.float64, device=x.device)
            elif tuple(t.shape) != (2,) or t.dtype != torch.float64 or t.device != x.device or not t.is_contiguous():
                raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"output 'norms' must be a contiguous float64 (2,) tensor on {x.device}")
            res["norms"] = t
        if flags or want_norms:
            check(lib.cpl_eval_batch_ex(ctypes.byref(self.desc()), B, p(x), p(mass), p(env_tag), p(res.get("g")),
                                        p(res.get("jac")), p(res.get("f")), p(res.get("grad")), p(res.get("norms")),
                                        flags, ctypes.c_void_p(s.cuda_stream)))
            return res
        check(lib.cpl_eval_batch(ctypes.byref(self.desc()), B, p(x), p(mass), p(env_tag), p(res.get("g")),
                                 p(res.get("jac")), p(res.get("f")), p(res.get("grad")),
                                 ctypes.c_void_p(s.cuda_stream)))
        return res

    def residual_norms(self, g, stream=None):
        """[max violation, sum of squared violations] of a device g batch (device tensor [2])."""
        import torch

        B = g.shape[0]
        out = torch.empty(2, dtype=torch.float64, device=g.device)
        s = stream if stream is not None else torch.cuda.current_stream(g.device)
        check(lib.cpl_residual_norms(ctypes.byref(self.desc()), B, ctypes.c_void_p(g.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream)))
        return out
