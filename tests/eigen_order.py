"""How far apart the two plausible Eigen builds of the reference lie (test infrastructure).

The reference's Eigen is unpinned.  Its Vector3d dot / squaredNorm / norm
reduce the three terms as
  * (a0 b0 + a1 b1) + a2 b2  — Eigen 3.3 with the default x86-64 SSE2 packets (the oracle's order,
    and the kernels'), or
  * a0 b0 + (a1 b1 + a2 b2)  — without packet math for a 3-vector (no vectorisation, or AVX, whose
    4-double packets are longer than a Vector3d): oracle/_build/libcpl_oracle_novec.so.
The orders meet in FrictionCone (F.dot(n) in both values and in t1 of the Jacobian,
src/Constraints/FrictionCone.cpp:39-40, 71), Superquadric's normal (the gradient's norm,
src/Superquadric.cpp:66-68) and the cost's squared norms (src/MinimizeCentroidalVariables.cpp:130-145).
`order_deviation` reports, per output class, how many entries differ and by how much: plain
relative |a - b| / |b|, and for the friction-cone values (which cancel when the cone is active) the
deviation relative to their un-cancelled terms.
"""
from __future__ import annotations

import numpy as np

import pyoracle

G_CLASSES = ("statics", "env", "normal", "cone0", "cone1")


def row_classes(prob, env):
    """Class name of every g row [m] (statics / env / normal / cone0 / cone1)."""
    _, m, _ = prob.get_nlp_info()
    cls = np.empty(m, dtype=object)
    cls[:6] = "statics"
    per = 6 if env != "none" else 2
    names = ("env", "normal", "normal", "normal", "cone0", "cone1") if env != "none" else ("cone0", "cone1")
    for r in range(6, m):
        cls[r] = names[(r - 6) % per]
    return cls


def cone_active(x, N, mu):
    """x with every contact's tangential force scaled onto the cone boundary |F_t| = mu F.n (the
    friction-cone value then cancels to ~0: the case where the reduction order shows most)."""
    x = np.array(x, dtype=np.float64, copy=True)
    for i in range(N):
        F = x[:, 3 + 9 * i: 6 + 9 * i]
        n = x[:, 9 + 9 * i: 12 + 9 * i]
        fn = (F * n).sum(1, keepdims=True)
        ft = F - fn * n
        nt = np.linalg.norm(ft, axis=1, keepdims=True)
        with np.errstate(all="ignore"):
            ft = np.where(nt > 0, ft / nt, 0.0) * (mu * np.abs(fn))
        x[:, 3 + 9 * i: 6 + 9 * i] = fn * n + ft
    return x


def _cone_scales(prob, x, env):
    """Un-cancelled magnitude of the two cone values per contact block (map order) [B, N, 2]."""
    N = len(prob.contact_names)
    order = prob.map_order
    mu = prob.GetMu()
    out = np.zeros((x.shape[0], N, 2))
    for k, i in enumerate(order):
        F = x[:, 3 + 9 * i: 6 + 9 * i]
        n = x[:, 9 + 9 * i: 12 + 9 * i]
        fabs = np.abs(F * n).sum(1)
        ft = np.linalg.norm(F - (F * n).sum(1, keepdims=True) * n, axis=1)
        out[:, k, 0] = fabs
        out[:, k, 1] = ft + mu * fabs
    return out


def _jac_cone1_scales(prob, x, env):
    """Un-cancelled magnitude of each friction-cone row-1 Jacobian entry [B, N, 6]
    (src/Constraints/FrictionCone.cpp:85-99: (sum of three products) / s * (-1/2) - mu * n_k or F_k),
    every difference inside replaced by the sum of its operands' magnitudes."""
    N = len(prob.contact_names)
    mu = prob.GetMu()
    out = np.zeros((x.shape[0], N, 6))
    for k, i in enumerate(prob.map_order):
        F = np.abs(x[:, 3 + 9 * i: 6 + 9 * i])
        n = np.abs(x[:, 9 + 9 * i: 12 + 9 * i])
        Fs = x[:, 3 + 9 * i: 6 + 9 * i]
        ns = x[:, 9 + 9 * i: 12 + 9 * i]
        t1 = (F * n).sum(1)
        t = F + n * t1[:, None]                          # |F_j - n_j t1| bounded
        s = np.linalg.norm(Fs - (Fs * ns).sum(1, keepdims=True) * ns, axis=1)
        tF = F * n                                       # t5, t6, t7
        for j in range(3):
            o1, o2 = [q for q in range(3) if q != j]
            aF = t[:, j] * (n[:, j] * n[:, j] + 1.0) * 2 + n[:, j] * n[:, o1] * t[:, o1] * 2 + n[:, j] * n[:, o2] * t[:, o2] * 2
            an = t[:, j] * (tF[:, o1] + tF[:, o2] + tF[:, j] * 2) * 2 + F[:, j] * n[:, o1] * t[:, o1] * 2 + \
                F[:, j] * n[:, o2] * t[:, o2] * 2
            with np.errstate(all="ignore"):
                out[:, k, j] = aF / s / 2 + mu * n[:, j]
                out[:, k, 3 + j] = an / s / 2 + mu * F[:, j]
    return out


def order_deviation(prob, env, x, mass=None, tag=None, got=None):
    """Per output class: entries, entries that differ between the two orders (bit level), the largest
    plain relative and absolute deviation, and (cone values) the largest deviation relative to the
    un-cancelled terms.  got: outputs to compare with the non-vectorised order instead of the oracle's
    SSE2 order (e.g. the GPU's, same inputs)."""
    desc = prob.desc()
    a = got if got is not None else pyoracle.eval_batch(desc, x, mass, tag, outputs=("g", "jac", "f"))
    b = pyoracle.eval_batch(desc, x, mass, tag, outputs=("g", "jac", "f"), variant="novec")
    rows = row_classes(prob, env)
    iRow, _ = pyoracle.structure(desc)
    jcls = rows[iRow]
    N = len(prob.contact_names)
    res = {}

    def stats(va, vb, scale=None):
        va, vb = np.asarray(va, dtype=np.float64), np.asarray(vb, dtype=np.float64)
        both = ~(np.isnan(va) | np.isnan(vb))
        diff = both & (va != vb)
        d = np.abs(va - vb)
        with np.errstate(all="ignore"):
            rel = np.where(diff, d / np.abs(vb), 0.0)
        s = {"entries": int(va.size), "differ": int(diff.sum()),
             "nan_mismatch": int((np.isnan(va) != np.isnan(vb)).sum()),
             "max_abs": float(d[diff].max()) if diff.any() else 0.0,
             "max_rel": float(rel[diff].max()) if diff.any() else 0.0}
        if scale is not None:
            with np.errstate(all="ignore"):
                sc = np.where(diff, d / scale, 0.0)
            s["max_rel_uncancelled"] = float(sc[diff].max()) if diff.any() else 0.0
        return s

    cs = _cone_scales(prob, x, env)
    for c in G_CLASSES:
        sel = rows == c
        if not sel.any():
            continue
        scale = None
        if c in ("cone0", "cone1"):
            scale = cs[:, :, 0 if c == "cone0" else 1]
        if c == "normal":  # n - n_env: cancels where the normal matches the surface's; scale |n| + |n_env|
            nsc = np.stack([np.linalg.norm(x[:, 9 + 9 * i: 12 + 9 * i], axis=1) for i in prob.map_order], axis=1)
            scale = np.repeat(nsc + 1.0, 3, axis=1)
        res["g_" + c] = stats(a["g"][:, sel], b["g"][:, sel], scale)
        jsel = jcls == c
        res["jac_" + c] = stats(a["jac"][:, jsel], b["jac"][:, jsel],
                                _jac_cone1_scales(prob, x, env).reshape(x.shape[0], -1) if c == "cone1" else None)
    if "f" in a:  # (a caller's outputs may carry g and the Jacobian only)
        res["f"] = stats(a["f"], b["f"])
    res["instances"] = int(x.shape[0])
    res["contacts"] = N
    return res


BINS = [0.0, 1e-16, 1e-15, 1e-14, 1e-13, 1e-12, 1e-11, 1e-10, 1e-9, 1e-8, np.inf]


def histogram(prob, env, x, mass=None, tag=None, got=None):
    """Per output class, the differing entries binned by plain relative deviation (edges BINS; the
    last bin holds the infinite ones: a value exactly 0 in one order and not in the other)."""
    desc = prob.desc()
    a = got if got is not None else pyoracle.eval_batch(desc, x, mass, tag, outputs=("g", "jac", "f"))
    b = pyoracle.eval_batch(desc, x, mass, tag, outputs=("g", "jac", "f"), variant="novec")
    rows = row_classes(prob, env)
    iRow, _ = pyoracle.structure(desc)
    jcls = rows[iRow]
    out = {}
    for key, va, vb in ([("g_" + c, a["g"][:, rows == c], b["g"][:, rows == c]) for c in G_CLASSES] +
                        [("jac_" + c, a["jac"][:, jcls == c], b["jac"][:, jcls == c]) for c in G_CLASSES] +
                        [("f", a["f"], b["f"])]):
        if va.size == 0:
            continue
        diff = (va != vb) & ~(np.isnan(va) | np.isnan(vb))
        with np.errstate(all="ignore"):
            rel = np.abs(va - vb)[diff] / np.abs(vb[diff])
        counts, _ = np.histogram(np.where(np.isinf(rel), 1e300, rel), bins=BINS[:-1] + [1e299, np.inf])
        out[key] = {"entries": int(va.size), "differ": int(diff.sum()), "counts": counts.tolist()}
    out["bin_edges"] = [str(e) for e in BINS]
    return out

