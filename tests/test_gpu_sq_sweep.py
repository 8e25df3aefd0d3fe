"""Superquadric parameter sweep on the GPU against the oracle (src/Superquadric.cpp:7-209).

The double-double power ladders run only when every P is an integer in [2, 64]; every other
exponent goes through cpow's other paths (integer exponents beyond the ladder, half-integers in
double-double, general exponents through the device's pow).  Sets covered:
  * the default Superquadric() (C = (0,0,10), R = P = (10,10,10); src/Superquadric.cpp:7-9);
  * P in {2, 3, 5} (odd P: negative bases give negative odd powers);
  * P in {2.5, 3.7} (half-integer and general: glibc gives NaN for a negative base, and so must we);
  * P = 80 (outside the ladder) and mixed per-axis P;
  * N = 32 (CPL_MAX_CONTACTS), Superquadric, Ground, mixed and no environment.
Parity policy: tests/parity_util.py (bit-exact off the pow-bearing entries, 1e-10 of the
conditioning-aware scale on them, NaN positions identical), and every pow-bearing entry off the three
normal-Jacobian diagonals within 1e-10 PLAIN relative error (asserted).  The diagonals themselves
are graded on the plain 1e-10 bound too wherever |ref| is above the rounding noise of their
un-cancelled terms (parity_util.plain_rel_diagonals: the count of graded entries outside the bound
and of the noise-floor entries is reported).  The plain relative-error histograms are written to
gpurun_out/sq_sweep_hist.json next to the scaled figure.
"""
import json
import os

import numpy as np
import pytest

import pyoracle
from parity_util import RTOL, check_outputs, plain_rel_diagonals, plain_rel_off_diagonals

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REPORT = {}


def _sq_problem(N, C, R, P, mu=0.5):
    from centroidalplanner_amd import CplProblem, Superquadric

    e = Superquadric()
    if C is not None:
        e.SetParameters(C, R, P)
    e.SetMu(mu)
    prob = CplProblem([f"contact{i + 1}" for i in range(N)], 80.0, e)
    prob.SetManipulationWrench([100.0, 0.0, 0.0, 0.0, 0.0, 100.0])
    return prob


def _sq_points(prob, B, seed, box=1.3):
    """p = C + R * U(-box, box) per axis (the surface lies at |(p-C)/R| <= 1), |p_k - C_k| >= 1e-3 R_k;
    F inside the cone around a unit n near the outward normal direction, random CoM and masses."""
    from parity_util import sq_params

    C, R, _ = sq_params(prob)
    N = len(prob.contact_names)
    rng = np.random.default_rng(seed)
    x = np.empty((B, prob.n))
    x[:, 0:3] = rng.uniform(-0.2, 0.2, (B, 3)) + np.array([0.0, 0.0, 1.0])
    for i in range(N):
        u = rng.uniform(-box, box, (B, 3))
        u = np.where(np.abs(u) < 1e-3, np.copysign(1e-3, u), u)
        p = C + R * u
        nv = rng.normal(size=(B, 3))
        nv /= np.linalg.norm(nv, axis=1, keepdims=True)
        F = rng.uniform(5.0, 200.0, (B, 1)) * nv + rng.normal(scale=10.0, size=(B, 3))
        x[:, 3 + 9 * i: 6 + 9 * i] = F
        x[:, 6 + 9 * i: 9 + 9 * i] = p
        x[:, 9 + 9 * i: 12 + 9 * i] = nv
    mass = rng.uniform(20.0, 150.0, B)
    return x, mass


def _run(prob, x, mass, tag=None):
    dev = torch.device("cuda:0")
    xt = torch.tensor(x, device=dev)
    mt = torch.tensor(mass, device=dev)
    tt = None if tag is None else torch.tensor(tag, device=dev)
    out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "f", "grad"))
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    ref = pyoracle.eval_batch(prob.desc(), x, mass, tag)
    return got, ref


def _summary(rep):
    keys = ("ok", "bitwise_frac", "nan_mismatch", "exact_violations", "max_scaled_err", "max_plain_rel_err",
            "plain_rel_hist", "tol_entries")
    return {k: {kk: rep[k][kk] for kk in keys} for k in ("g", "jac")}


SETS = {
    "default": (None, None, None),
    "P2": ([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [2.0, 2.0, 2.0]),
    "P3": ([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [3.0, 3.0, 3.0]),
    "P5": ([0.1, -0.2, 1.0], [0.3, 0.5, 2.0], [5.0, 5.0, 5.0]),
    "P2.5": ([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [2.5, 2.5, 2.5]),
    "P3.7": ([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [3.7, 3.7, 3.7]),
    "P80": ([0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [80.0, 80.0, 80.0]),
    "Pmixed": ([0.2, 0.0, 1.0], [0.4, 0.3, 1.5], [4.0, 6.5, 10.0]),
}


@pytest.mark.parametrize("name", list(SETS))
@pytest.mark.parametrize("N", [4, 8])
def test_superquadric_parameter_sweep(name, N):
    C, R, P = SETS[name]
    prob = _sq_problem(N, C, R, P)
    x, mass = _sq_points(prob, 1501, 17 + N)
    got, ref = _run(prob, x, mass)
    rep = check_outputs(prob, "superquadric", x, got, ref, raise_on_fail=False)
    plain = plain_rel_off_diagonals(prob, "superquadric", x, got, ref)
    diag = plain_rel_diagonals(prob, "superquadric", x, got, ref)
    _REPORT[f"{name}/N{N}"] = dict(_summary(rep), plain_off_diagonal=plain, plain_diagonal=diag)
    assert all(rep[k]["ok"] for k in rep), (name, N, rep)
    # the north-star bound as a PLAIN relative error on every pow-bearing entry off the diagonals
    assert plain["g"] <= RTOL and plain["jac"] <= RTOL, (name, N, plain)
    if name in ("P2.5", "P3.7"):  # negative bases: NaN (glibc pow), at the same positions
        assert np.isnan(ref["jac"]).any()


@pytest.mark.parametrize("env", ["superquadric", "ground", "mixed", "none"])
def test_max_contacts(env):
    """N = CPL_MAX_CONTACTS = 32 (records of 291 / 198 / 1350 doubles with an environment)."""
    from centroidalplanner_amd.workload import generate, make_problem

    prob = make_problem(32, env)
    x, mass, tag = generate(32, env, 203, 321)
    got, ref = _run(prob, x, mass, tag)
    rep = check_outputs(prob, env, x, got, ref, tag, raise_on_fail=False)
    plain = plain_rel_off_diagonals(prob, env, x, got, ref, tag)
    diag = plain_rel_diagonals(prob, env, x, got, ref, tag)
    _REPORT[f"N32/{env}"] = dict(_summary(rep), plain_off_diagonal=plain, plain_diagonal=diag)
    assert all(rep[k]["ok"] for k in rep), (env, rep)
    assert plain["g"] <= RTOL and plain["jac"] <= RTOL, (env, plain)


def test_write_report():
    """Writes the histogram report (runs after the cases above in file order)."""
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sq_sweep_hist.json"), "w") as fh:
        json.dump(_REPORT, fh, indent=1, sort_keys=True)
