"""CPU tests of the C-ABI: the library loads, exports every symbol include/*.h declares, and its
host half (descriptor defaults and validation, dimensions, Jacobian structure, bounds) agrees with
the oracle's independent assembly and the reference's documented behaviour.  No device calls."""
import ctypes
import glob
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle
from centroidalplanner_amd import _abi
from centroidalplanner_amd.workload import make_problem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for mt in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s+(cpl_[a-z_0-9]+)\s*\(", src, flags=re.M):
            names.add(mt.group(1))
    return names


def test_exports_every_declared_symbol():
    declared = _declared_functions()
    assert len(declared) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = declared - exported
    assert not missing, f"declared but not exported: {missing}"
    assert declared <= set(_abi.SIGNATURES), "ctypes mirror lacks a declared function"


def test_abi_version_and_layout():
    assert _abi.lib.cpl_abi_version() == _abi.ABI_VERSION
    assert _abi.lib.cpl_desc_sizeof() == ctypes.sizeof(_abi.ProblemDesc)
    assert _abi.lib.cpl_status_string(0) == b"ok"


def test_desc_defaults_match_reference_constructors():
    d = _abi.ProblemDesc()
    _abi.check(_abi.lib.cpl_desc_init(ctypes.byref(d), 4, _abi.ENV_GROUND, 100.0))
    assert d.mass == 100.0 and list(d.gravity) == [0.0, 0.0, -9.81]      # CentroidalStatics.cpp:14-15
    assert list(d.wrench) == [0.0] * 6 and d.mu == 1.0 and d.ground_z == 0.0
    assert list(d.sq_C) == [0, 0, 10] and list(d.sq_R) == [10] * 3 and list(d.sq_P) == [10] * 3
    assert d.W_com == 1.0 and list(d.com_ref) == [0, 0, 1]                # MinimizeCentroidalVariables.cpp:11-25
    assert d.W_p[0] == 1.0 and d.W_F[3] == 1.0 and d.F_thr[2] == 0.0
    assert d.F_lb[0][0] == -1000.0 and d.n_ub[3][2] == 1000.0             # Variable3D.cpp:12-13


@pytest.mark.parametrize("call,msg", [
    (lambda d: _abi.lib.cpl_desc_init(ctypes.byref(d), 4, 1, 0.0), "Invalid robot mass"),
    (lambda d: _abi.lib.cpl_desc_init(ctypes.byref(d), 0, 1, 1.0), "n_contacts"),
    (lambda d: _abi.lib.cpl_desc_init(ctypes.byref(d), 33, 1, 1.0), "n_contacts"),
    (lambda d: _abi.lib.cpl_desc_set_mu(ctypes.byref(d), 0.0), "Invalid friction coefficient"),
])
def test_validation_errors(call, msg):
    d = _abi.ProblemDesc()
    _abi.check(_abi.lib.cpl_desc_init(ctypes.byref(d), 4, 1, 50.0))
    st = call(d)
    assert st == _abi.ERR_INVALID_ARGUMENT
    assert msg in _abi.lib.cpl_last_error().decode()


def test_superquadric_and_bounds_validation():
    d = _abi.ProblemDesc()
    _abi.check(_abi.lib.cpl_desc_init(ctypes.byref(d), 2, 2, 50.0))
    v = lambda *a: (ctypes.c_double * 3)(*a)  # noqa: E731
    assert _abi.lib.cpl_desc_set_superquadric(ctypes.byref(d), v(0, 0, 1), v(1, 0, 1), v(2, 2, 2)) == 1
    assert b"radii" in _abi.lib.cpl_last_error()
    assert _abi.lib.cpl_desc_set_superquadric(ctypes.byref(d), v(0, 0, 1), v(1, 1, 1), v(2, 1.5, 2)) == 1
    assert b"curvatures" in _abi.lib.cpl_last_error()
    assert _abi.lib.cpl_desc_set_superquadric(ctypes.byref(d), v(0, 0, 1), v(1, 1, 1), v(2, 2, 2)) == 0
    assert _abi.lib.cpl_desc_set_bounds(ctypes.byref(d), 1, 0, v(0, 0, 1), v(1, 1, 0)) == 1
    assert b"Inconsistent bounds" in _abi.lib.cpl_last_error()
    assert _abi.lib.cpl_desc_set_bounds(ctypes.byref(d), 1, 5, v(0, 0, 0), v(1, 1, 1)) == _abi.ERR_OUT_OF_RANGE


def test_duplicate_contact_names_rejected():
    d = _abi.ProblemDesc()
    _abi.check(_abi.lib.cpl_desc_init(ctypes.byref(d), 3, 1, 50.0))
    arr = (ctypes.c_char_p * 3)(b"a", b"b", b"a")
    assert _abi.lib.cpl_desc_set_contact_names(ctypes.byref(d), arr, 3) == _abi.ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("N", [1, 2, 4, 8, 10, 11, 16, 32])
@pytest.mark.parametrize("env", ["ground", "superquadric", "none", "mixed"])
def test_structure_and_bounds_match_oracle_assembly(N, env):
    prob = make_problem(N, env)
    d = prob.desc()
    assert prob.get_nlp_info() == pyoracle.dims(d)
    iR, jC = prob.get_structure()
    oR, oC = pyoracle.structure(d)
    assert np.array_equal(iR, oR) and np.array_equal(jC, oC)
    rp = prob.get_row_ptr()
    assert rp[0] == 0 and rp[-1] == len(iR) and np.array_equal(np.diff(rp), np.bincount(iR, minlength=prob.m))
    # RowMajor CSR: columns strictly ascending within each row
    for r in range(prob.m):
        cols = jC[rp[r]:rp[r + 1]]
        assert np.all(np.diff(cols) > 0)
    for a, b in zip(prob.get_bounds_info(), pyoracle.bounds(d)):
        assert np.array_equal(a, b)


def test_dims_match_survey_probe():
    """N=1 -> 12/12/48; N=4 -> 39/30/174 (no env 39/14/114); N=8 -> 75/54/342;
    N=16 -> 147/102/678 (verified there on the shim-compiled reference)."""
    assert make_problem(1, "ground").get_nlp_info() == (12, 12, 48)
    assert make_problem(4, "ground").get_nlp_info() == (39, 30, 174)
    assert make_problem(4, "none").get_nlp_info() == (39, 14, 114)
    assert make_problem(8, "superquadric").get_nlp_info() == (75, 54, 342)
    assert make_problem(16, "mixed").get_nlp_info() == (147, 102, 678)


def test_map_order_diverges_from_vector_order():
    """std::map order puts "contact10" before "contact2" (src/CplProblem.cpp:42 vs :21)."""
    prob = make_problem(12, "ground")
    names = prob.contact_names
    assert [names[i] for i in prob.map_order] == sorted(names)
    assert prob.map_order[:4] == [0, 9, 10, 11]


def test_bounds_cone_rows_one_sided():
    prob = make_problem(3, "ground")
    xl, xu, gl, gu = prob.get_bounds_info()
    for k in range(3):
        base = 6 + 6 * k
        assert list(gl[base: base + 4]) == [0.0] * 4 and list(gu[base: base + 4]) == [0.0] * 4
        assert list(gl[base + 4: base + 6]) == [-_abi.INF] * 2 and list(gu[base + 4: base + 6]) == [0.0] * 2


@pytest.mark.parametrize("nw,m,ok", [(128, 30, True), (128, 31, False), (47, 47, True), (10, 11, False)])
def test_kkt_qd_solve_rejects_what_does_not_fit_before_launch(nw, m, ok):
    """cpl_kkt_qd_solve checks its LDS image (nw^2 + nw + 2m + m nw doubles <= 160 KiB) and m <= nw up
    front: an oversized system is CPL_ERR_UNSUPPORTED (m > nw: invalid), never a failed launch.  With
    batch 0 a fitting system returns before touching the GPU."""
    fn = _abi.lib.cpl_kkt_qd_solve
    rc = fn(0, nw, m, *([None] * 12))
    if ok:
        assert rc == 0
    else:
        assert rc in (_abi.ERR_UNSUPPORTED, _abi.ERR_INVALID_ARGUMENT)
        if m <= nw:
            assert rc == _abi.ERR_UNSUPPORTED and "LDS" in _abi.lib.cpl_last_error().decode()


def test_solver_rejects_bad_jacobian_regularization_before_any_gpu_call():
    """cpl_solve_options.jacobian_regularization: 0 / 1 only (CPL_ERR_INVALID_ARGUMENT otherwise), and
    IPOPT's form needs the augmented system (nw + m unknowns) to fit the workgroup KKT kernel (<= 128):
    the 8-contact problem's does not — CPL_ERR_UNSUPPORTED, checked before the solver touches the GPU."""
    from centroidalplanner_amd.workload import solve_problem

    for nc, jr, want in ((4, 2, _abi.ERR_INVALID_ARGUMENT), (8, 1, _abi.ERR_UNSUPPORTED)):
        prob = solve_problem(nc).GetCplProblem()
        o = _abi.SolveOptions()
        _abi.lib.cpl_solve_options_default(ctypes.byref(o))
        assert o.jacobian_regularization == 0
        o.jacobian_regularization = jr
        h = ctypes.c_void_p()
        d = prob.desc()
        assert _abi.lib.cpl_solver_create(ctypes.byref(d), 4, ctypes.byref(o), ctypes.byref(h)) == want
        assert not h.value
