"""centroidalplanner_amd — MI355X-native batched NLP-callback engine for CentroidalPlanner.

The hot path (IFOPT's eval_g / eval_jac_g / eval_f / eval_grad_f over many independent
CentroidalPlanner instances) runs as hand-written HIP kernels for gfx950 behind the C-ABI in
``include/cpl_mi355x.h``; this package is the host-side mirror of the reference's problem API.
Importing it loads ``libcpl_mi355x.so`` and fails loudly if it has not been built.
"""
from ._abi import (ENV_GROUND, ENV_MIXED, ENV_NONE, ENV_SUPERQUADRIC, INF, MAX_CONTACTS, CplError, InvalidArgument,
                   OutOfRange, ProblemDesc)
from .planner import CentroidalPlanner, CoMPlanner, ContactValues, Solution
from .problem import CplProblem, EnvironmentClass, Ground, MixedEnvironment, Superquadric

__all__ = [
    "CentroidalPlanner",
    "CoMPlanner",
    "Solution",
    "ContactValues",
    "CplProblem",
    "EnvironmentClass",
    "Ground",
    "Superquadric",
    "MixedEnvironment",
    "ProblemDesc",
    "CplError",
    "InvalidArgument",
    "OutOfRange",
    "ENV_NONE",
    "ENV_GROUND",
    "ENV_SUPERQUADRIC",
    "ENV_MIXED",
    "INF",
    "MAX_CONTACTS",
]
