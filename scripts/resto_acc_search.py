"""Search for solves that reach IPOPT's RestoreAcceptablePoint branch (a failed restoration phase with a
backup acceptable point), in the compiled restatement (oracle/cpl_solve_host.c): TestBasic-like
scenarios with randomised parameters and start points, acceptable_tol off (-1), over a few tol values.
Every solve whose restoration phase fails at a feasible point is printed with the err0 history of its
regular iterates (CPLO_TRACE), from which an acceptable_tol that stores a backup point before the
failing restoration phase (and does not stop the solve earlier) is chosen.  CPU only.

python scripts/resto_acc_search.py [count] [seed] [--exact] [--host] > out.jsonl
(--exact: the exact-Hessian mode too; --host: batch_ipm.py over the oracle at the first restoring
acceptable_tol of every hit)
"""
import json
import os
import sys
import warnings
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from resto_cases import NAMES, make  # noqa: E402


def draw(rng):
    """A TestBasic-like scenario's parameters (JSON-able; make() builds the planner)."""
    kind = int(rng.integers(0, 4))
    nc = int(rng.integers(1, 5))
    P = {"kind": ["ground", "ground", "superquadric", "com"][kind], "contacts": NAMES[:nc] if kind < 3 else NAMES,
         "mass": float(rng.uniform(20.0, 150.0)), "wrench": (rng.normal(0.0, 60.0, 6) * (rng.uniform() < 0.7)).tolist()}
    if kind == 3:
        P["mu"] = float(rng.uniform(0.2, 1.0))
        P["positions"] = [(rng.uniform(-1.2, 1.2, 3) * np.array([1, 1, 0.1])).tolist() for _ in NAMES]
        P["lifting"] = NAMES[int(rng.integers(0, 4))] if rng.uniform() < 0.7 else None
        P["thresholds"] = [float(rng.uniform(0.0, 40.0)) for _ in NAMES]
    else:
        if kind == 2:
            P["sq"] = [(rng.uniform(-0.2, 0.2, 3) + np.array([0, 0, 1.0])).tolist(), rng.uniform(0.2, 0.6, 3).tolist(),
                       rng.choice([2.0, 4.0, 10.0], 3).tolist()]
        else:
            P["ground_z"] = float(rng.uniform(-0.2, 0.3))
        P["mu"] = float(rng.uniform(0.2, 1.0))
        P["com_weight"] = float(rng.choice([0.0, 1.0, 2.0, 10.0]))
        P["force_weight"] = float(rng.choice([0.0, 1e-3, 1.0]))
        P["pos_bounds"] = []
        for _ in P["contacts"]:
            lo = rng.uniform(-0.6, 0.0, 3)
            P["pos_bounds"].append([lo.tolist(), (lo + rng.uniform(0.2, 1.5, 3)).tolist()])
    return P


def case(seed):
    """(parameters, the planner, x0) of a seed: x = 0 or a perturbed start."""
    rng = np.random.default_rng(seed)
    P = draw(rng)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        cpl = make(P)
        x0 = cpl.GetCplProblem().get_starting_point()
    if rng.uniform() < 0.5:
        x0 = x0 + rng.normal(0.0, 1.0, x0.shape) * rng.choice([0.01, 1.0, 100.0])
    return P, cpl, x0


def host(prob, x0, tol, acceptable_tol, hessian):
    """batch_ipm.py over the CPU oracle's callbacks: (status, iterations, objective, restored)."""
    import torch

    import centroidalplanner_amd.batch_ipm as bi
    from centroidalplanner_amd.batch_ipm import batch_ipm_solve
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_batch_solve import OracleBatchEvaluator

    log = []
    bi._DEBUG_EVENT = lambda name, mask: log.append(name)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([prob.desc().mass])), tol=tol,
                                max_iter=3000, evaluator=OracleBatchEvaluator(prob, 1), hessian=hessian,
                                acceptable_tol=acceptable_tol)
    finally:
        bi._DEBUG_EVENT = None
    return int(h.status[0]), int(h.iterations[0]), float(h.objective[0]), "restore_acceptable_point" in log


def one(args):
    import pyoracle

    seed, tol, hessian = args
    P, cpl, x0 = case(seed)
    prob = cpl.GetCplProblem()
    if hessian == "exact" and P["kind"] == "superquadric":
        return None
    pyoracle.set_acceptable_tol(-1.0)
    pyoracle.resto_fail_events()
    try:
        r = pyoracle.solve(prob.desc(), x0, prob.desc().mass, max_iter=3000, tol=tol, hessian=hessian)
    except ValueError:
        return None
    ev = pyoracle.resto_fail_events()
    out = {"seed": seed, "tol": tol, "hessian": hessian, "status": pyoracle.STATUS_NAMES[r["status"]],
           "iterations": r["iterations"], "restorations": r["restorations"], "resto_failed": ev[0], "restored_at": []}
    if ev[0]:  # the acceptable_tol values at which the failure restores a backup acceptable point instead
        for at in np.logspace(-10, 2, 49):
            pyoracle.set_acceptable_tol(at)
            pyoracle.resto_fail_events()
            r2 = pyoracle.solve(prob.desc(), x0, prob.desc().mass, max_iter=3000, tol=tol, hessian=hessian)
            if pyoracle.resto_fail_events()[1]:
                out["restored_at"].append({"acceptable_tol": float(at), "iterations": r2["iterations"],
                                           "objective": r2["objective"]})
        pyoracle.set_acceptable_tol(-1.0)
        if out["restored_at"] and HOST:  # the host restatement at the smallest restoring acceptable_tol
            ra = out["restored_at"][0]
            st, it, obj, restored = host(prob, x0, tol, ra["acceptable_tol"], hessian)
            out["host"] = {"status": st, "iterations": it, "objective": obj, "restored": restored}
        out["params"] = P
    return out


HOST = "--host" in sys.argv


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    count = int(argv[0]) if argv else 200
    seed0 = int(argv[1]) if len(argv) > 1 else 0
    hessians = ("limited-memory", "exact") if "--exact" in sys.argv else ("limited-memory",)
    jobs = [(seed0 + i, tol, h) for i in range(count) for tol in (1e-8, 1e-6, 1e-4) for h in hessians]
    hits = 0
    with Pool(8) as pool:
        for r in pool.imap_unordered(one, jobs, chunksize=4):
            if r is None:
                continue
            if r["resto_failed"]:
                hits += 1
                print(json.dumps(r), flush=True)
    print(json.dumps({"solves": len(jobs), "resto_failed_solves": hits}), flush=True)


if __name__ == "__main__":
    main()
