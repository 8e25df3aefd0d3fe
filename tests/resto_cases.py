"""TestBasic-like scenarios from a parameter dict (scripts/resto_acc_search.py draws them): the cases
whose solves call IPOPT's restoration phase at an almost feasible point (tests/golden/resto_acc_cases.json)."""
import numpy as np

NAMES = ["contact1", "contact2", "contact3", "contact4"]


def make(P):
    """The planner of parameters P (kind: ground / superquadric / com; TestBasic.cpp's setters)."""
    from centroidalplanner_amd import CentroidalPlanner, CoMPlanner, Ground, Superquadric

    if P["kind"] == "com":
        cpl = CoMPlanner(NAMES, P["mass"])
        cpl.SetMu(P["mu"])
        for c, p in zip(NAMES, P["positions"]):
            cpl.SetContactPosition(c, np.array(p))
        if P["lifting"]:
            cpl.SetLiftingContact(P["lifting"])
        for c, t in zip(NAMES, P["thresholds"]):
            cpl.SetForceThreshold(c, t)
        return cpl
    if P["kind"] == "superquadric":
        env = Superquadric()
        env.SetParameters(*(np.array(v) for v in P["sq"]))
    else:
        env = Ground()
        env.SetGroundZ(P["ground_z"])
    env.SetMu(P["mu"])
    cpl = CentroidalPlanner(P["contacts"], P["mass"], env)
    cpl.SetCoMWeight(P["com_weight"])
    cpl.SetForceWeight(P["force_weight"])
    for c, (lo, up) in zip(P["contacts"], P["pos_bounds"]):
        cpl.SetPosBounds(c, np.array(lo), np.array(up))
    cpl.SetManipulationWrench(np.array(P["wrench"]))
    return cpl
