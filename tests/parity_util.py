"""Comparison policy of the GPU path against the oracle (test infrastructure).

Policy:
  * every entry that does not depend on a data-dependent pow (statics, friction cone, Ground,
    cost) must be bit-identical (+0.0 == -0.0), NaN positions identical;
  * Superquadric entries (environment value / Jacobian / normal value / normal Jacobian) go through
    pow, where the GPU uses a correctly rounded double-double power and glibc misrounds ~0.1 % of
    calls by one ulp.  They must satisfy |gpu - ref| <= RTOL * scale with RTOL = 1e-10 (the
    north-star tolerance), where scale = |ref| for every entry except the three normal-Jacobian
    diagonals, whose expanded (C-p)^2 numerator cancels catastrophically
    (src/Superquadric.cpp:98-100, 152-154, 206-208): there scale is the magnitude of the
    un-cancelled terms, |lead / S^1.5| * sum|E terms|, evaluated in float64 from the same inputs.
"""
from __future__ import annotations

import numpy as np

RTOL = 1e-10

def contact_offsets(N, has_env, map_order):
    """jac offset of the per-contact block of map position k, and g offset."""
    statics = 6 + 15 * N
    cj = 27 if has_env else 12
    cg = 6 if has_env else 2
    return [(statics + cj * k, 6 + cg * k, map_order[k]) for k in range(N)]


def sq_entry_mask(N, map_order, nnz, m, sq_instances):
    """Boolean masks [B, nnz] / [B, m] of the pow-bearing entries of Superquadric instances."""
    jm = np.zeros(nnz, dtype=bool)
    gm = np.zeros(m, dtype=bool)
    for jo, go, _ in contact_offsets(N, True, map_order):
        jm[jo: jo + 15] = True      # env row (3) + normal rows (12)
        gm[go: go + 4] = True       # env value + normal value
    B = len(sq_instances)
    return np.where(sq_instances[:, None], jm[None, :], False), np.where(sq_instances[:, None], gm[None, :], False)


def diag_scale(x, N, map_order, C, R, P):
    """[B, N, 3] conditioning scale of the normal-Jacobian diagonals (per contact, map order)."""
    B = x.shape[0]
    out = np.zeros((B, N, 3))
    with np.errstate(all="ignore"):
        for k in range(N):
            i = map_order[k]
            p = x[:, 6 + 9 * i: 9 + 9 * i]
            d = p - C
            inv = 1.0 / (d * d)
            p2P = np.abs(d) ** (2 * P)
            Rm2 = R ** (-(2 * P))
            Rp2 = R ** (2 * P)
            T = Rm2 * inv * P * P * p2P
            Dg = P * P * R ** (-2 * P) * p2P * inv
            for a in range(3):
                b, c = [q for q in range(3) if q != a]
                lead = P[a] * R[a] ** (-P[a]) * np.abs(d[:, a]) ** P[a] * (P[a] - 1.0)
                for q in range(3):
                    lead = lead * (1.0 if q == a else Rm2[q]) * inv[:, q]
                S = T[:, b] + T[:, c] + Dg[:, a]
                terms = (np.abs(C[b] * C[b]) + p[:, b] ** 2 + 2 * np.abs(C[b] * p[:, b])) * P[c] ** 2 * p2P[:, c] * Rp2[b] \
                    + (np.abs(C[c] * C[c]) + p[:, c] ** 2 + 2 * np.abs(C[c] * p[:, c])) * P[b] ** 2 * p2P[:, b] * Rp2[c]
                out[:, k, a] = np.abs(lead / S ** 1.5) * terms
    return out


def compare(got, want, exact_mask=None, scale=None, rtol=RTOL):
    """Returns (ok, stats).  exact_mask: entries that must be bit-identical (default: all)."""
    got = np.asarray(got)
    want = np.asarray(want)
    nan_g, nan_w = np.isnan(got), np.isnan(want)
    stats = {"n": got.size, "nan_mismatch": int((nan_g != nan_w).sum())}
    both = ~(nan_g | nan_w)
    eq = (got == want) | (nan_g & nan_w)
    stats["bitwise_frac"] = float(eq.mean()) if got.size else 1.0
    if exact_mask is None:
        exact_mask = np.ones(got.shape, dtype=bool)
    bad_exact = exact_mask & ~eq
    stats["exact_violations"] = int(bad_exact.sum())
    tol_mask = ~exact_mask & both
    if scale is None:
        scale = np.abs(want)
    with np.errstate(all="ignore"):  # equal infinities (P = 80 overflows) count as equal, not inf - inf
        err = np.where(tol_mask & ~eq, np.abs(got - want), 0.0)
    with np.errstate(all="ignore"):
        rel = np.where(tol_mask & (scale > 0), err / np.where(scale > 0, scale, 1.0), np.where(err > 0, np.inf, 0.0))
    stats["max_scaled_err"] = float(rel.max()) if rel.size else 0.0
    # plain relative error |gpu - ref| / |ref| of the tolerance entries, next to the scaled one:
    # histogram over decades (bitwise equal, < 1e-15, < 1e-13, < 1e-12, < 1e-10, >= 1e-10)
    with np.errstate(all="ignore"):
        plain = np.where(tol_mask, err / np.where(np.abs(want) > 0, np.abs(want), 1.0), 0.0)
        plain = np.where(tol_mask & (want == 0) & (err > 0), np.inf, plain)
    tv = plain[tol_mask & ~eq]
    stats["tol_entries"] = int(tol_mask.sum())
    stats["plain_rel_hist"] = {
        "bitwise": int((tol_mask & eq).sum()),
        "lt1e-15": int((tv < 1e-15).sum()),
        "lt1e-13": int(((tv >= 1e-15) & (tv < 1e-13)).sum()),
        "lt1e-12": int(((tv >= 1e-13) & (tv < 1e-12)).sum()),
        "lt1e-10": int(((tv >= 1e-12) & (tv < 1e-10)).sum()),
        "ge1e-10": int((tv >= 1e-10).sum()),
    }
    stats["max_plain_rel_err"] = float(tv.max()) if tv.size else 0.0
    ok = stats["nan_mismatch"] == 0 and stats["exact_violations"] == 0 and stats["max_scaled_err"] <= rtol
    return ok, stats


def g_scale(x, N, map_order, got_ref, C, R, P, sq_inst):
    """Scale of the Superquadric g entries: env value = sum pow - 1 -> sum|pow| + 1; normal value
    n - n_env -> |n| + |n_env|."""
    scale = np.abs(got_ref).copy()
    with np.errstate(all="ignore"):
        for jo, go, i in contact_offsets(N, True, map_order):
            p = x[:, 6 + 9 * i: 9 + 9 * i]
            nv = x[:, 9 + 9 * i: 12 + 9 * i]
            d = p - C
            s_env = (np.abs(d / R) ** P).sum(1) + 1.0
            j = P / R ** P * np.abs(d) ** (P - 1)
            en = j / np.linalg.norm(j, axis=1, keepdims=True)
            scale[:, go] = np.where(sq_inst, np.maximum(scale[:, go], s_env), scale[:, go])
            for a in range(3):
                s_n = np.abs(nv[:, a]) + np.abs(en[:, a])
                scale[:, go + 1 + a] = np.where(sq_inst, np.maximum(scale[:, go + 1 + a], s_n), scale[:, go + 1 + a])
    return scale


def sq_params(prob):
    """(C, R, P) of the problem's Superquadric (the template's current parameters)."""
    d = prob.desc()
    return np.array(d.sq_C[:]), np.array(d.sq_R[:]), np.array(d.sq_P[:])


def plain_rel_off_diagonals(prob, env, x, got, ref, tag=None):
    """Plain relative error |gpu - ref| / |ref| of every pow-bearing entry EXCEPT the three
    normal-Jacobian diagonals of each Superquadric contact (whose expanded numerators cancel,
    src/Superquadric.cpp:98-100,152-154,206-208, and are graded on the scale of check_outputs):
    the environment value / normal residual entries of g and the environment-gradient and
    off-diagonal normal-Jacobian entries of jac.  Returns {"g": max, "jac": max, "entries": count,
    "hist": decades} (NaN positions are compared by check_outputs, skipped here)."""
    from centroidalplanner_amd import ENV_SUPERQUADRIC

    N = len(prob.contact_names)
    n, m, nnz = prob.get_nlp_info()
    B = x.shape[0]
    sq_inst = (np.ones(B, dtype=bool) if env == "superquadric" else
               (tag == ENV_SUPERQUADRIC) if env == "mixed" else np.zeros(B, dtype=bool))
    out = {"entries": 0, "g": 0.0, "jac": 0.0,
           "hist": {"bitwise": 0, "lt1e-15": 0, "lt1e-13": 0, "lt1e-12": 0, "lt1e-10": 0, "ge1e-10": 0}}
    if not sq_inst.any():  # no Superquadric contact rows in this layout: no pow-bearing entries
        return out
    jm, gm = sq_entry_mask(N, prob.map_order, nnz, m, sq_inst)
    for jo, _, _ in contact_offsets(N, True, prob.map_order):
        for a in range(3):
            jm[:, jo + 3 + 4 * a + a] = False  # the diagonal of normal-Jacobian row a
    for k, mask in (("g", gm), ("jac", jm)):
        gv, rv = np.asarray(got[k]), np.asarray(ref[k])
        sel = mask & ~(np.isnan(gv) | np.isnan(rv))
        with np.errstate(all="ignore"):
            err = np.where(sel & (gv != rv), np.abs(gv - rv), 0.0)
            rel = np.where(err > 0, err / np.where(np.abs(rv) > 0, np.abs(rv), 0.0), 0.0)
        rel = np.where(sel & (err > 0) & (rv == 0), np.inf, rel)
        v = rel[sel]
        out[k] = float(v.max()) if v.size else 0.0
        out["entries"] += int(sel.sum())
        nz = v[v > 0]
        h = out["hist"]
        h["bitwise"] += int((v == 0).sum())
        h["lt1e-15"] += int((nz < 1e-15).sum())
        h["lt1e-13"] += int(((nz >= 1e-15) & (nz < 1e-13)).sum())
        h["lt1e-12"] += int(((nz >= 1e-13) & (nz < 1e-12)).sum())
        h["lt1e-10"] += int(((nz >= 1e-12) & (nz < 1e-10)).sum())
        h["ge1e-10"] += int((nz >= 1e-10).sum())
    return out


NOISE_ULPS = 8.0  # |ref| at or below this many ulps of the un-cancelled terms' magnitude: rounding noise


def plain_rel_diagonals(prob, env, x, got, ref, tag=None):
    """The three normal-Jacobian diagonals of each Superquadric contact graded on the PLAIN relative
    error |gpu - ref| / |ref| wherever |ref| is not itself rounding noise of its un-cancelled terms
    (|ref| > NOISE_ULPS * eps * diag_scale: the expanded (C - p)^2 numerator cancels,
    src/Superquadric.cpp:98-100, 152-154, 206-208).  Returns {"graded": count, "noise": count of the
    entries at the noise floor (graded on the scale of check_outputs only), "max": max plain relative
    error over the graded entries, "outside": graded entries above RTOL, "hist": decades, and
    "outside_ref_over_scale": |ref| / scale of the entries above RTOL (at most 32)}."""
    from centroidalplanner_amd import ENV_SUPERQUADRIC

    N = len(prob.contact_names)
    B = x.shape[0]
    sq_inst = (np.ones(B, dtype=bool) if env == "superquadric" else
               (tag == ENV_SUPERQUADRIC) if env == "mixed" else np.zeros(B, dtype=bool))
    out = {"graded": 0, "noise": 0, "max": 0.0, "outside": 0, "outside_ref_over_scale": [],
           "hist": {"bitwise": 0, "lt1e-15": 0, "lt1e-13": 0, "lt1e-12": 0, "lt1e-10": 0, "ge1e-10": 0}}
    if not sq_inst.any():
        return out
    ds = diag_scale(x, N, prob.map_order, *sq_params(prob))
    gv, rv = np.asarray(got["jac"]), np.asarray(ref["jac"])
    eps = np.finfo(np.float64).eps
    for kk, (jo, _, _) in enumerate(contact_offsets(N, True, prob.map_order)):
        for a in range(3):
            col = jo + 3 + 4 * a + a
            g, r, s = gv[:, col], rv[:, col], ds[:, kk, a]
            fin = sq_inst & ~(np.isnan(g) | np.isnan(r)) & np.isfinite(s)
            with np.errstate(all="ignore"):
                noise = fin & ~(np.abs(r) > NOISE_ULPS * eps * s)
                sel = fin & ~noise
                err = np.where(sel & (g != r), np.abs(g - r), 0.0)
                rel = np.where(err > 0, err / np.where(np.abs(r) > 0, np.abs(r), 1.0), 0.0)
            out["noise"] += int(noise.sum())
            out["graded"] += int(sel.sum())
            v = rel[sel]
            if v.size:
                out["max"] = max(out["max"], float(v.max()))
            nz = v[v > 0]
            h = out["hist"]
            h["bitwise"] += int((v == 0).sum())
            h["lt1e-15"] += int((nz < 1e-15).sum())
            h["lt1e-13"] += int(((nz >= 1e-15) & (nz < 1e-13)).sum())
            h["lt1e-12"] += int(((nz >= 1e-13) & (nz < 1e-12)).sum())
            h["lt1e-10"] += int(((nz >= 1e-12) & (nz < 1e-10)).sum())
            h["ge1e-10"] += int((nz >= 1e-10).sum())
            bad = sel & (rel > RTOL)
            out["outside"] += int(bad.sum())
            with np.errstate(all="ignore"):
                ros = np.abs(r[bad]) / s[bad]
            out["outside_ref_over_scale"] += [float(t) for t in ros[: 32 - len(out["outside_ref_over_scale"])]]
    return out


def plain_rel_g_graded(prob, env, x, got, ref, tag=None):
    """The Superquadric g entries (environment value sum pow - 1, normal residual n - n_env: both cancel
    near the surface) graded on the PLAIN relative error wherever |ref| is above the rounding noise of
    their un-cancelled terms (|ref| > NOISE_ULPS * eps * g_scale).  Returns {"graded", "noise", "max",
    "outside": graded entries above RTOL, "outside_err_ulps": their |gpu - ref| in units of eps *
    g_scale (at most 32), "outside_ref_over_scale", "hist"}."""
    from centroidalplanner_amd import ENV_SUPERQUADRIC

    N = len(prob.contact_names)
    n, m, nnz = prob.get_nlp_info()
    B = x.shape[0]
    sq_inst = (np.ones(B, dtype=bool) if env == "superquadric" else
               (tag == ENV_SUPERQUADRIC) if env == "mixed" else np.zeros(B, dtype=bool))
    out = {"graded": 0, "noise": 0, "max": 0.0, "outside": 0, "outside_err_ulps": [], "outside_ref_over_scale": [],
           "hist": {"bitwise": 0, "lt1e-15": 0, "lt1e-13": 0, "lt1e-12": 0, "lt1e-10": 0, "ge1e-10": 0}}
    if not sq_inst.any():
        return out
    _, gm = sq_entry_mask(N, prob.map_order, nnz, m, sq_inst)
    gv, rv = np.asarray(got["g"]), np.asarray(ref["g"])
    scale = g_scale(x, N, prob.map_order, rv, *sq_params(prob), sq_inst)
    eps = np.finfo(np.float64).eps
    with np.errstate(all="ignore"):
        fin = gm & ~(np.isnan(gv) | np.isnan(rv)) & np.isfinite(scale)
        noise = fin & ~(np.abs(rv) > NOISE_ULPS * eps * scale)
        sel = fin & ~noise
        err = np.where(sel & (gv != rv), np.abs(gv - rv), 0.0)
        rel = np.where(err > 0, err / np.where(np.abs(rv) > 0, np.abs(rv), 1.0), 0.0)
    out["noise"] = int(noise.sum())
    out["graded"] = int(sel.sum())
    v = rel[sel]
    out["max"] = float(v.max()) if v.size else 0.0
    nz = v[v > 0]
    h = out["hist"]
    h["bitwise"] = int((v == 0).sum())
    h["lt1e-15"] = int((nz < 1e-15).sum())
    h["lt1e-13"] = int(((nz >= 1e-15) & (nz < 1e-13)).sum())
    h["lt1e-12"] = int(((nz >= 1e-13) & (nz < 1e-12)).sum())
    h["lt1e-10"] = int(((nz >= 1e-12) & (nz < 1e-10)).sum())
    h["ge1e-10"] = int((nz >= 1e-10).sum())
    bad = sel & (rel > RTOL)
    out["outside"] = int(bad.sum())
    with np.errstate(all="ignore"):
        out["outside_err_ulps"] = [float(t) for t in (err[bad] / (eps * scale[bad]))[:32]]
        out["outside_ref_over_scale"] = [float(t) for t in (np.abs(rv[bad]) / scale[bad])[:32]]
    return out


def check_outputs(prob, env, x, got, ref, tag=None, raise_on_fail=True):
    """Apply the policy above to every output; returns {output: stats}; raises AssertionError
    (raise_on_fail=False: every output is checked and stats["ok"] says whether it passed)."""
    from centroidalplanner_amd import ENV_SUPERQUADRIC

    SQ = sq_params(prob)
    N = len(prob.contact_names)
    n, m, nnz = prob.get_nlp_info()
    B = x.shape[0]
    if env == "superquadric":
        sq_inst = np.ones(B, dtype=bool)
    elif env == "mixed":
        sq_inst = tag == ENV_SUPERQUADRIC
    else:
        sq_inst = np.zeros(B, dtype=bool)
    jm, gm = sq_entry_mask(N, prob.map_order, nnz, m, sq_inst)
    report = {}
    for k in got:
        if k == "jac":
            scale = np.abs(ref[k]).copy()
            if sq_inst.any():
                ds = diag_scale(x, N, prob.map_order, *SQ)
                for kk, (jo, _, _) in enumerate(contact_offsets(N, True, prob.map_order)):
                    for a in range(3):
                        col = jo + 3 + 4 * a + a
                        scale[:, col] = np.where(sq_inst, np.maximum(scale[:, col], ds[:, kk, a]), scale[:, col])
            ok, st = compare(got[k], ref[k], exact_mask=~jm, scale=scale)
        elif k == "g":
            scale = g_scale(x, N, prob.map_order, ref[k], *SQ, sq_inst) if sq_inst.any() else None
            ok, st = compare(got[k], ref[k], exact_mask=~gm, scale=scale)
        else:
            ok, st = compare(got[k], ref[k])
        st["ok"] = bool(ok)
        report[k] = st
        if raise_on_fail:
            assert ok, f"{env} N={N} B={B} output {k}: {st}"
    return report
