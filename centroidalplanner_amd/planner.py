"""Facade API: cpl::CentroidalPlanner and cpl::CoMPlanner (host side of the batched engine).

Mirrors include/CentroidalPlanner/CentroidalPlanner.h and CoMPlanner.h: same method names, same
argument meaning, same validation and error kinds (std::invalid_argument -> InvalidArgument,
std::runtime_error -> CplError(ERR_RUNTIME)).  Solve() runs the batched interior-point solve loop on
one instance (centroidalplanner_amd.solver: IPOPT's method with IFOPT's defaults — limited-memory
Hessian, max_iter 3000, tol 1e-8) over the GPU callbacks; like the reference's persistent problem,
the variables keep the last solution between solves (warm start).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _abi
from ._abi import CplError, InvalidArgument
from .problem import CplProblem, EnvironmentClass
from .solver import solve


@dataclass
class ContactValues:
    """include/CentroidalPlanner/Ifopt/Types.h:8-13; pycpl's read-only names force / position /
    normal (bindings/python/pyCpl.cpp:34-37) are aliases of the C++ member names."""

    force_value: np.ndarray
    position_value: np.ndarray
    normal_value: np.ndarray

    @property
    def force(self) -> np.ndarray:
        return self.force_value

    @property
    def position(self) -> np.ndarray:
        return self.position_value

    @property
    def normal(self) -> np.ndarray:
        return self.normal_value


def _eigen_row(v) -> str:
    """Eigen's default IOFormat for a row vector (what `ss << v.transpose()` prints): every
    coefficient in the stream's default format (%g, 6 significant digits), right-aligned to the
    widest coefficient, separated by one space."""
    cells = [f"{float(c):g}" for c in np.asarray(v, dtype=np.float64).reshape(-1)]
    w = max((len(c) for c in cells), default=0)
    return " ".join(c.rjust(w) for c in cells)


@dataclass
class Solution:
    """include/CentroidalPlanner/Ifopt/Types.h:15-21 (contact_values_map iterates in name order);
    pycpl's ``com`` (bindings/python/pyCpl.cpp:39-42) aliases com_sol, and ``repr`` is operator<<."""

    com_sol: np.ndarray
    contact_values_map: Dict[str, ContactValues] = field(default_factory=dict)
    success: bool = True
    message: str = ""
    iterations: int = 0  # the interior-point iterations the solve took (IPOPT's iteration count)
    fallback: bool = False  # not converged and the last iterate infeasible: the best feasible iterate instead
    nan_jacobian_at_start: int = 0  # NaN Jacobian entries at the start point, taken as 0 (solver.py)

    @property
    def com(self) -> np.ndarray:
        return self.com_sol

    def __str__(self) -> str:  # operator<< (src/CplProblem.cpp:321-344)
        lines = [f"CoM: {_eigen_row(self.com_sol)}"]
        lines += [f"F_{k}: {_eigen_row(v.force_value)}" for k, v in self.contact_values_map.items()]
        lines += [f"p_{k}: {_eigen_row(v.position_value)}" for k, v in self.contact_values_map.items()]
        lines += [f"n_{k}: {_eigen_row(v.normal_value)}" for k, v in self.contact_values_map.items()]
        return "\n".join(lines) + "\n"

    __repr__ = __str__  # pyCpl.cpp:38 binds __repr__ to operator<<


def _v3(v) -> np.ndarray:
    return np.asarray(v, dtype=np.float64).reshape(3)


class CentroidalPlanner:
    """src/CentroidalPlanner.cpp"""

    def __init__(self, contact_names: Sequence[str], robot_mass: float, env: Optional[EnvironmentClass]):
        if robot_mass <= 0.0:  # src/CentroidalPlanner.cpp:12-15
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid robot mass")
        self._contact_names = [str(c) for c in contact_names]
        self._robot_mass = float(robot_mass)
        self._env = env
        self._cpl_problem = CplProblem(self._contact_names, self._robot_mass, env)
        self.evaluator = None  # None: GPU callbacks; tests may inject the oracle
        # IFOPT's IpoptSolver defaults the reference runs with (src/CentroidalPlanner.cpp:22-29)
        self.solver_tol = 1e-8
        self.solver_max_iter = 3000
        self.solver_hessian = "limited-memory"
        # a rank-deficient constraint Jacobian: "pivot" (the engine's default, delta_c on R's small
        # pivots) or "ipopt" (IPOPT's (2,2)-block regularisation, cpl_solve_options.jacobian_regularization)
        self.solver_jacobian_regularization = "pivot"
        # src/CentroidalPlanner.cpp:26 SetOption("derivative_test", "first-order"): IPOPT checks the
        # first derivatives at the start point of every solve; the report lands here
        self.solver_derivative_test = "first-order"
        self.last_derivative_report = None

    # ---- Solve (src/CentroidalPlanner.cpp:22-34) ------------------------------------------
    def Solve(self) -> Solution:
        res = solve(self._cpl_problem, evaluator=self.evaluator, tol=self.solver_tol, max_iter=self.solver_max_iter,
                    hessian=self.solver_hessian, jacobian_regularization=self.solver_jacobian_regularization,
                    derivative_test=self.solver_derivative_test if self.evaluator is None else "none")
        self.last_derivative_report = res.derivative_report
        sol = self._cpl_problem.GetSolution()
        out = Solution(com_sol=sol["com"], success=res.success, message=res.status, iterations=res.iterations,
                       fallback=res.fallback, nan_jacobian_at_start=res.nan_jacobian_at_start)
        for name, cv in sol["contact_values_map"].items():
            out.contact_values_map[name] = ContactValues(cv["force"], cv["position"], cv["normal"])
        return out

    # ---- validation helpers ------------------------------------------------------------------
    def HasContact(self, contact_name: str) -> bool:  # :359-370
        return contact_name in self._contact_names

    def _check_contact(self, contact_name: str) -> None:
        if not self.HasContact(contact_name):
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, f"Invalid contact name: '{contact_name}'")

    @staticmethod
    def _check_weight(w: float) -> None:
        if w < 0.0:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid weight")

    def GetCplProblem(self) -> CplProblem:
        return self._cpl_problem

    # ---- bounds (:37-124) ---------------------------------------------------------------------
    def SetForceBounds(self, contact_name, force_lb, force_ub):
        self._check_contact(contact_name)
        self._cpl_problem.SetForceBounds(contact_name, force_lb, force_ub)

    def GetForceBounds(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetForceBounds(contact_name)

    def SetPosBounds(self, contact_name, pos_lb, pos_ub):
        self._check_contact(contact_name)
        self._cpl_problem.SetPosBounds(contact_name, pos_lb, pos_ub)

    def GetPosBounds(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetPosBounds(contact_name)

    def SetNormalBounds(self, contact_name, normal_lb, normal_ub):  # protected in the reference
        self._check_contact(contact_name)
        self._cpl_problem.SetNormalBounds(contact_name, normal_lb, normal_ub)

    def GetNormalBounds(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetNormalBounds(contact_name)

    # ---- references and weights (:126-303) ----------------------------------------------------
    def SetPosRef(self, contact_name, pos_ref):
        self._check_contact(contact_name)
        self._cpl_problem.SetPosRef(contact_name, pos_ref)

    def GetPosRef(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetPosRef(contact_name)

    def SetForceRef(self, contact_name, force_ref):
        self._check_contact(contact_name)
        self._cpl_problem.SetForceRef(contact_name, force_ref)

    def GetForceRef(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetForceRef(contact_name)

    def SetCoMRef(self, com_ref):
        self._cpl_problem.SetCoMRef(com_ref)

    def GetCoMRef(self):
        return self._cpl_problem.GetCoMRef()

    def SetCoMWeight(self, W_CoM):
        self._check_weight(W_CoM)
        self._cpl_problem.SetCoMWeight(W_CoM)

    def GetCoMWeight(self):
        return self._cpl_problem.GetCoMWeight()

    def SetPosWeight(self, W_p):
        self._check_weight(W_p)
        self._cpl_problem.SetPosWeight(W_p)

    def GetPosWeight(self) -> Dict[str, float]:
        return {c: self._cpl_problem.GetContactPosWeight(c) for c in sorted(self._contact_names, key=str.encode)}

    def SetContactPosWeight(self, contact_name, W_p):
        self._check_contact(contact_name)
        self._check_weight(W_p)
        self._cpl_problem.SetContactPosWeight(contact_name, W_p)

    def GetContactPosWeight(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetContactPosWeight(contact_name)

    def SetForceWeight(self, W_F):
        self._check_weight(W_F)
        self._cpl_problem.SetForceWeight(W_F)

    def GetForceWeight(self) -> Dict[str, float]:
        return {c: self._cpl_problem.GetContactForceWeight(c) for c in sorted(self._contact_names, key=str.encode)}

    def SetContactForceWeight(self, contact_name, W_F):
        self._check_contact(contact_name)
        self._check_weight(W_F)
        self._cpl_problem.SetContactForceWeight(contact_name, W_F)

    def GetContactForceWeight(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetContactForceWeight(contact_name)

    def SetManipulationWrench(self, wrench_manip):
        self._cpl_problem.SetManipulationWrench(wrench_manip)

    def GetManipulationWrench(self):
        return self._cpl_problem.GetManipulationWrench()

    def GetMu(self):
        return self._cpl_problem.GetMu()

    # ---- force threshold (:324-356) -----------------------------------------------------------
    def SetForceThreshold(self, contact_name, F_thr):
        self._check_contact(contact_name)
        if F_thr < 0.0:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid force threshold")
        lb, ub = self._cpl_problem.GetForceBounds(contact_name)
        # Eigen operator!= : true when any coefficient differs (src/CentroidalPlanner.cpp:340)
        if np.any(lb != 0.0) and np.any(ub != 0.0):
            self._cpl_problem.SetForceThreshold(contact_name, F_thr)

    def GetForceThreshold(self, contact_name):
        self._check_contact(contact_name)
        return self._cpl_problem.GetForceThreshold(contact_name)


class CoMPlanner:
    """src/CoMPlanner.cpp — privately inherits CentroidalPlanner with env = nullptr."""

    def __init__(self, contact_names: Sequence[str], robot_mass: float):
        self._cp = CentroidalPlanner(contact_names, robot_mass, None)
        self._contact_names = [str(c) for c in contact_names]
        self._F_thr_map: Dict[str, float] = {}
        self._cp.SetPosWeight(0.0)
        self._cp.SetForceWeight(0.0)
        for c in self._contact_names:  # :13-23
            self.SetContactNormal(c, [0.0, 0.0, 1.0])
            self._F_thr_map[c] = self._cp.GetForceThreshold(c)

    @property
    def evaluator(self):
        return self._cp.evaluator

    @evaluator.setter
    def evaluator(self, ev):
        self._cp.evaluator = ev

    def SetLiftingContact(self, contact_name):  # :27-37
        self._F_thr_map[contact_name] = self._cp.GetForceThreshold(contact_name)
        self._cp.SetForceThreshold(contact_name, 0.0)
        self._cp.SetForceBounds(contact_name, np.zeros(3), np.zeros(3))

    def GetLiftingContacts(self) -> List[str]:  # :40-56
        out = []
        for c in self._contact_names:
            lb, ub = self._cp.GetForceBounds(c)
            if np.all(lb == 0.0) and np.all(ub == 0.0):
                out.append(c)
        return out

    def IsLiftingContact(self, contact_name) -> bool:
        return contact_name in self.GetLiftingContacts()

    def ResetLiftingContact(self, contact_name):  # :74-88
        if not self.IsLiftingContact(contact_name):
            raise CplError(_abi.ERR_RUNTIME, f"'{contact_name}' is not a lifting contact.")
        self._cp.SetForceBounds(contact_name, -1e3 * np.ones(3), 1e3 * np.ones(3))
        self._cp.SetForceThreshold(contact_name, self._F_thr_map[contact_name])

    def SetContactPosition(self, contact_name, pos_ref):  # :91-97
        self._cp.SetPosBounds(contact_name, pos_ref, pos_ref)

    def GetContactPosition(self, contact_name):  # :100-111
        lb, ub = self._cp.GetPosBounds(contact_name)
        if np.any(lb != ub):
            raise CplError(_abi.ERR_RUNTIME, f"Contact position for '{contact_name}' not set")
        return lb

    def SetContactNormal(self, contact_name, n_ref):  # :114-129
        self._cp._check_contact(contact_name)
        self._cp.SetNormalBounds(contact_name, n_ref, n_ref)

    def GetContactNormal(self, contact_name):  # :132-143
        lb, ub = self._cp.GetNormalBounds(contact_name)
        if np.any(lb != ub):
            raise CplError(_abi.ERR_RUNTIME, f"Contact normal for '{contact_name}' not set")
        return lb

    def SetMu(self, mu):  # :146-156
        if mu <= 0.0:
            raise InvalidArgument(_abi.ERR_INVALID_ARGUMENT, "Invalid friction coefficient")
        self._cp.GetCplProblem().SetMu(mu)

    # using CentroidalPlanner::... (include/CentroidalPlanner/CoMPlanner.h:67-78)
    def Solve(self):
        return self._cp.Solve()

    def SetCoMWeight(self, w):
        self._cp.SetCoMWeight(w)

    def GetCoMWeight(self):
        return self._cp.GetCoMWeight()

    def SetPosWeight(self, w):
        self._cp.SetPosWeight(w)

    def GetPosWeight(self):
        return self._cp.GetPosWeight()

    def SetForceWeight(self, w):
        self._cp.SetForceWeight(w)

    def GetForceWeight(self):
        return self._cp.GetForceWeight()

    def SetCoMRef(self, r):
        self._cp.SetCoMRef(r)

    def GetCoMRef(self):
        return self._cp.GetCoMRef()

    def SetForceThreshold(self, c, F_thr):
        self._cp.SetForceThreshold(c, F_thr)

    def GetForceThreshold(self, c):
        return self._cp.GetForceThreshold(c)

    def GetMu(self):
        return self._cp.GetMu()

    def GetCplProblem(self) -> CplProblem:
        return self._cp.GetCplProblem()
