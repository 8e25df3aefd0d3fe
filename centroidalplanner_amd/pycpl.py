"""pycpl — the reference's Python module surface (bindings/python/pyCpl.cpp:12-70) over this package.

    import centroidalplanner_amd.pycpl as cpl      # or, unchanged from the reference's examples:
    import centroidal_planner.pycpl as cpl

Same class and attribute names as the pybind11 module: EnvironmentClass (GetMu / SetMu), Ground
(SetGroundZ), Superquadric (SetParameters / GetParameters), ContactValues (force / position /
normal), Solution (com / contact_values_map, __repr__ = operator<<), CentroidalPlanner (the eleven
methods pyCpl.cpp:44-58 binds) and CoMPlanner (a CentroidalPlanner in Python, as pybind11 declares
it with `base`: its own six methods of pyCpl.cpp:61-69 plus the base's).  Solve() runs the native
solve engine on the GPU (centroidalplanner_amd.solver).
"""
from __future__ import annotations

from abc import ABCMeta

from .planner import CentroidalPlanner as _CentroidalPlanner
from .planner import CoMPlanner as _CoMPlanner
from .planner import ContactValues, Solution
from .problem import EnvironmentClass, Ground, Superquadric


class CentroidalPlanner(_CentroidalPlanner, metaclass=ABCMeta):
    """pyCpl.cpp:44-58: CentroidalPlanner(contact_names, robot_mass, env)."""


class CoMPlanner(_CoMPlanner):
    """pyCpl.cpp:61-69: py::class_<CoMPlanner>(m, "CoMPlanner", base) — the base's bound methods are
    callable on a CoMPlanner too."""

    def SetPosRef(self, contact_name, pos_ref):
        self._cp.SetPosRef(contact_name, pos_ref)

    def SetPosBounds(self, contact_name, pos_lb, pos_ub):
        self._cp.SetPosBounds(contact_name, pos_lb, pos_ub)

    def SetForceBounds(self, contact_name, force_lb, force_ub):
        self._cp.SetForceBounds(contact_name, force_lb, force_ub)

    def SetManipulationWrench(self, wrench_manip):
        self._cp.SetManipulationWrench(wrench_manip)


# pyCpl.cpp:61 declares CentroidalPlanner as CoMPlanner's base: isinstance(com, CentroidalPlanner) holds
# (the C++ CoMPlanner inherits privately and the Python one delegates, so it is a virtual subclass)
CentroidalPlanner.register(CoMPlanner)

__all__ = ["EnvironmentClass", "Ground", "Superquadric", "ContactValues", "Solution", "CentroidalPlanner",
           "CoMPlanner"]
