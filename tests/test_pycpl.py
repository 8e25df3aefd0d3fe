"""The reference's Python surface (bindings/python/pyCpl.cpp:12-70) and its example script
(examples/python/test.py:7-42, written in Python 3: the script's only Python-2 construct is its
first `print`): the module path `centroidal_planner.pycpl`, pycpl's attribute names, and the two
example scenarios solved from the planners' defaults (x = 0, src/Variable3D.cpp:8-10).

`oracle` runs the solve loop over the CPU restatement's callbacks (test infrastructure); `gpu` runs
the product path (the native engine), exactly what `planner.Solve()` does in the example."""
import numpy as np
import pytest

import pyoracle
import centroidal_planner.pycpl as cpl


class _Oracle:
    def __init__(self, problem):
        self.problem = problem

    def eval_batch(self, X):
        return pyoracle.eval_batch(self.problem.desc(), np.atleast_2d(X), outputs=("g", "jac", "f", "grad"),
                                   nthreads=1)


def _backend(planner, backend):
    if backend == "oracle":
        planner.evaluator = _Oracle(planner.GetCplProblem())


BACKENDS = [pytest.param("oracle"), pytest.param("gpu", marks=pytest.mark.gpu)]


def test_module_surface():
    """Every class and attribute pyCpl.cpp binds exists under its pycpl name."""
    for name in ("EnvironmentClass", "Ground", "Superquadric", "ContactValues", "Solution", "CentroidalPlanner",
                 "CoMPlanner"):
        assert hasattr(cpl, name), name
    for meth in ("GetMu", "SetMu"):
        assert hasattr(cpl.Ground(), meth)
    assert hasattr(cpl.Ground(), "SetGroundZ")
    assert hasattr(cpl.Superquadric(), "SetParameters") and hasattr(cpl.Superquadric(), "GetParameters")
    base = ("Solve", "SetCoMWeight", "SetPosWeight", "SetForceWeight", "SetCoMRef", "SetPosRef",
            "SetForceThreshold", "SetPosBounds", "SetForceBounds", "SetManipulationWrench", "GetForceThreshold")
    pl = cpl.CentroidalPlanner(["a", "b"], 20.0, cpl.Ground())
    for meth in base:
        assert callable(getattr(pl, meth)), meth
    com = cpl.CoMPlanner(["a", "b"], 20.0)
    for meth in base + ("SetLiftingContact", "ResetLiftingContact", "SetContactPosition", "GetContactPosition",
                        "SetContactNormal", "SetMu"):
        assert callable(getattr(com, meth)), meth
    assert isinstance(com, cpl.CentroidalPlanner)  # pyCpl.cpp:61: CentroidalPlanner is CoMPlanner's base
    assert not isinstance(pl, cpl.CoMPlanner)


def test_solution_repr_is_operator_shift():
    """Solution.__repr__ = operator<< (src/CplProblem.cpp:321-344): CoM, then F_, p_, n_ of every
    contact in name order, each vector as Eigen prints a row (%g, right-aligned to the widest)."""
    cv = cpl.ContactValues(np.array([1.0, -2.5, 30.0]), np.array([0.1, 0.2, 0.0]), np.array([0.0, 0.0, 1.0]))
    sol = cpl.Solution(np.array([0.0, -0.5, 1.0]), {"c1": cv, "c2": cv})
    assert sol.com is sol.com_sol
    assert cv.force is cv.force_value and cv.position is cv.position_value and cv.normal is cv.normal_value
    assert repr(sol) == ("CoM:    0 -0.5    1\n"
                         "F_c1:    1 -2.5   30\nF_c2:    1 -2.5   30\n"
                         "p_c1: 0.1 0.2   0\np_c2: 0.1 0.2   0\n"
                         "n_c1: 0 0 1\nn_c2: 0 0 1\n")
    assert str(sol) == repr(sol)


@pytest.mark.parametrize("backend", BACKENDS)
def test_example_centroidal_planner(backend):
    """examples/python/test.py:7-18: two contacts 'micio' / 'miao', mass 20, Ground at z = 0.1,
    every other setting at its default, Solve() from x = 0."""
    env = cpl.Ground()
    env.SetGroundZ(0.1)
    contacts = ["micio", "miao"]
    mass = 20.0
    planner = cpl.CentroidalPlanner(contacts, mass, env)
    _backend(planner, backend)
    sol = planner.Solve()
    text = repr(sol)
    assert text.startswith("CoM: ") and "F_miao:" in text and "n_micio:" in text
    assert list(sol.contact_values_map) == ["miao", "micio"]  # std::map order
    assert sol.success, sol.message
    Fz = sum(v.force[2] for v in sol.contact_values_map.values())
    assert Fz == pytest.approx(mass * 9.81, abs=1e-6)
    for v in sol.contact_values_map.values():
        assert v.position[2] == pytest.approx(0.1, abs=1e-6)
        assert v.normal[2] == pytest.approx(1.0, abs=1e-6)


@pytest.mark.parametrize("backend", BACKENDS)
def test_example_com_planner(backend):
    """examples/python/test.py:21-42: four contacts, mass 100, mu 0.5, CoM reference (0.2, 0.2, 1),
    contacts at (+-1, +-1, 0), c_3 and c_4 lifting."""
    contacts = ["c_1", "c_2", "c_3", "c_4"]
    mass, mu = 100.0, 0.5
    com_pl = cpl.CoMPlanner(contacts, mass)
    com_pl.SetMu(mu)
    com_pl.SetCoMRef([0.2, 0.2, 1.0])
    com_pl.SetContactPosition("c_1", [1.0, 1.0, 0.0])
    com_pl.SetContactPosition("c_2", [-1.0, 1.0, 0.0])
    com_pl.SetContactPosition("c_3", [1.0, -1.0, 0.0])
    com_pl.SetContactPosition("c_4", [-1.0, -1.0, 0.0])
    com_pl.SetLiftingContact("c_3")
    com_pl.SetLiftingContact("c_4")
    _backend(com_pl, backend)
    sol = com_pl.Solve()
    assert sol.success, sol.message
    F = {k: v.force for k, v in sol.contact_values_map.items()}
    assert np.abs(F["c_3"]).max() <= 1e-6 and np.abs(F["c_4"]).max() <= 1e-6  # lifted: zero force bounds
    Fsum = sum(F.values())
    assert Fsum == pytest.approx([0.0, 0.0, mass * 9.81], abs=1e-6)
    T = sum(np.cross(v.position - sol.com, v.force) for v in sol.contact_values_map.values())
    assert T == pytest.approx(np.zeros(3), abs=1e-4)
