"""CPU tests of the oracle (the CPU restatement used as parity checker).

* known-answer: a second, independent restatement in plain Python of the reference's formulas for
  one Ground contact and for the statics / cost blocks, bit-compared with the oracle;
* derivatives: central finite differences of g and f against the oracle's Jacobian / gradient for
  every environment (the analytic blocks are derivatives, not merely self-consistent);
* NaN semantics the reference has at degenerate points (SURVEY.md §7 hard part 2).
"""
import math

import numpy as np
import pytest

import pyoracle
from centroidalplanner_amd import CplProblem, Ground
from centroidalplanner_amd.workload import generate, make_problem


def dot(a, b):  # Eigen 3.3 Vector3d redux: (a0 b0 + a1 b1) + a2 b2
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def test_known_answer_ground_two_contacts():
    env = Ground()
    env.SetGroundZ(0.05)
    env.SetMu(0.6)
    prob = CplProblem(["b_foot", "a_foot"], 70.0, env)   # map order: a_foot (index 1), then b_foot (0)
    prob.SetManipulationWrench([1.5, -2.0, 3.0, 0.25, -0.5, 0.75])
    prob.SetForceThreshold("a_foot", 12.0)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, prob.n)
    out = pyoracle.eval_batch(prob.desc(), x[None], np.array([70.0]))
    g, jac = out["g"][0], out["jac"][0]
    c = x[0:3]
    F = [x[3 + 9 * i: 6 + 9 * i] for i in range(2)]
    p = [x[6 + 9 * i: 9 + 9 * i] for i in range(2)]
    nv = [x[9 + 9 * i: 12 + 9 * i] for i in range(2)]
    order = [1, 0]
    # statics values, CentroidalStatics.cpp:37-61
    v = [0.0] * 6
    for i in order:
        d = [p[i][k] - c[k] for k in range(3)]
        cr = [d[1] * F[i][2] - d[2] * F[i][1], d[2] * F[i][0] - d[0] * F[i][2], d[0] * F[i][1] - d[1] * F[i][0]]
        for k in range(3):
            v[k] += F[i][k]
            v[3 + k] += cr[k]
    w = [1.5, -2.0, 3.0, 0.25, -0.5, 0.75]
    v = [v[k] - w[k] for k in range(6)]
    mg = [70.0 * 0.0, 70.0 * 0.0, 70.0 * -9.81]
    v = [v[k] + mg[k] for k in range(3)] + v[3:]
    assert list(g[:6]) == v
    # per contact in map order: env, normal, cone (Ground.cpp, EnvironmentNormal.cpp, FrictionCone.cpp)
    thr = {1: 12.0, 0: 0.0}
    for k, i in enumerate(order):
        base = 6 + 6 * k
        assert g[base] == p[i][2] - 0.05
        assert list(g[base + 1: base + 4]) == [nv[i][0] - 0.0, nv[i][1] - 0.0, nv[i][2] - 1.0]
        t1 = dot(F[i], nv[i])
        tang = [F[i][q] - dot(nv[i], F[i]) * nv[i][q] for q in range(3)]
        assert g[base + 4] == -t1 + thr[i]
        assert g[base + 5] == math.sqrt(dot(tang, tang)) - 0.6 * t1
    # statics Jacobian rows 0-2 and the CoM block (CentroidalStatics.cpp:90-136)
    N = 2
    assert list(jac[: 3 * N]) == [1.0] * (3 * N)
    a31 = 0.0
    a32 = 0.0
    for i in order:
        a31 -= F[i][2]
        a32 -= -F[i][1]
    row3 = jac[3 * N: 3 * N + 2 + 4 * N]
    assert row3[0] == a31 and row3[1] == a32
    for i in range(N):  # column (vector) order
        assert list(row3[2 + 4 * i: 6 + 4 * i]) == [-(p[i][2] - c[2]), p[i][1] - c[1], F[i][2], -F[i][1]]
    # one cone Jacobian row-1 entry, FrictionCone.cpp:85
    i = order[0]
    n0, n1, n2 = nv[i]
    F0, F1, F2 = F[i]
    t1 = dot(F[i], nv[i])
    t2, t3, t4 = F0 - n0 * t1, F1 - n1 * t1, F2 - n2 * t1
    e = (t2 * (n0 * n0 - 1.0) * 2.0 + n0 * n1 * t3 * 2.0 + n0 * n2 * t4 * 2.0) * 1.0 / math.sqrt(
        t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - 0.6 * n0
    cone = 6 + 15 * N + 27 * 0 + 15
    assert jac[cone + 6] == e
    # cost, MinimizeCentroidalVariables.cpp:124-192 (defaults: W = 1, refs 0, CoM ref (0,0,1))
    val = 0.0
    for i in order:
        val += 0.5 * 1.0 * dot(p[i], p[i]) + 0.5 * 1.0 * dot(F[i], F[i])
    dc = [c[0], c[1], c[2] - 1.0]
    val += 0.5 * 1.0 * dot(dc, dc)
    assert out["f"][0] == val
    grad = out["grad"][0]
    assert list(grad[:3]) == [1.0 * dc[0], 1.0 * dc[1], 1.0 * dc[2]]
    assert list(grad[9:12]) == [0.0, 0.0, 0.0]


def test_known_answer_superquadric_values():
    """GetEnvironmentValue / GetEnvironmentJacobian / GetNormalValue (src/Superquadric.cpp:40-69) with
    glibc pow through Python's math.pow."""
    prob = make_problem(1, "superquadric")
    x = np.zeros(prob.n)
    x[0:3] = [0.01, -0.02, 1.1]
    x[3:6] = [10.0, -20.0, 300.0]
    p = [0.27, -0.11, 0.93]
    x[6:9] = p
    x[9:12] = [0.1, 0.2, 0.97]
    out = pyoracle.eval_batch(prob.desc(), x[None], np.array([100.0]))
    C, R, P = [0.0, 0.0, 1.0], [0.3, 0.3, 10.0], [10.0, 10.0, 10.0]
    val = 0.0
    for k in range(3):
        val += math.pow((p[k] - C[k]) / R[k], P[k])
    val -= 1.0
    j = [P[k] / math.pow(R[k], P[k]) * math.pow(p[k] - C[k], P[k] - 1) for k in range(3)]
    nrm = math.sqrt(dot(j, j))
    g = out["g"][0]
    assert g[6] == val
    assert list(g[7:10]) == [x[9 + k] - (-j[k] / nrm) for k in range(3)]
    assert list(out["jac"][0][6 + 15 + 0: 6 + 15 + 3]) == j


@pytest.mark.parametrize("env,N", [("ground", 3), ("superquadric", 3), ("none", 4), ("mixed", 4)])
def test_finite_differences(env, N):
    prob = make_problem(N, env)
    d = prob.desc()
    x, mass, tag = generate(N, env, 4, 321)
    n, m, nnz = prob.get_nlp_info()
    iR, jC = prob.get_structure()
    out = pyoracle.eval_batch(d, x, mass, tag)
    for b in range(4):
        J = np.zeros((m, n))
        J[iR, jC] = out["jac"][b]
        h = 1e-6 * np.maximum(1.0, np.abs(x[b]))
        P = np.repeat(x[b][None], 2 * n, axis=0)
        P[np.arange(n), np.arange(n)] += h
        P[n + np.arange(n), np.arange(n)] -= h
        o = pyoracle.eval_batch(d, P, np.full(2 * n, mass[b]), None if tag is None else np.full(2 * n, tag[b]))
        fdJ = ((o["g"][:n] - o["g"][n:]) / (2 * h[:, None])).T
        scale = np.maximum(1.0, np.abs(J)) * np.maximum(1.0, np.abs(out["g"][b]))[:, None]
        assert np.abs(fdJ - J).max() <= 1e-4 * scale.max(), np.abs(fdJ - J).max()
        assert (np.abs(fdJ - J) / scale).max() < 1e-6
        fdg = (o["f"][:n] - o["f"][n:]) / (2 * h)
        assert (np.abs(fdg - out["grad"][b]) / np.maximum(1.0, np.abs(out["f"][b]))).max() < 1e-7


def test_nan_positions_at_degenerate_points():
    """x = 0: every cone row-1 Jacobian entry is 0/0 (src/Constraints/FrictionCone.cpp:85-87,97-99);
    on the superquadric, p_k = C_k gives 0*inf in the normal-Jacobian diagonal (src/Superquadric.cpp:98)."""
    prob = make_problem(4, "ground")
    out = pyoracle.eval_batch(prob.desc(), np.zeros((1, prob.n)))
    jac = out["jac"][0]
    nan = np.isnan(jac)
    assert nan.sum() == 4 * 6                       # 6 row-1 cone entries per contact
    assert not np.isnan(out["g"][0]).any()
    sq = make_problem(1, "superquadric")
    x = np.zeros(sq.n)
    x[3:6] = [1.0, 2.0, 3.0]
    x[6:9] = [0.0, 0.05, 1.0]                        # p_x = C_x, p_z = C_z
    x[9:12] = [0.0, 0.0, 1.0]
    o = pyoracle.eval_batch(sq.desc(), x[None])
    nj = o["jac"][0][6 + 15 + 3: 6 + 15 + 15].reshape(3, 4)[:, :3]
    assert np.isnan(nj[0, 0])
