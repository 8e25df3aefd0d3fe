"""What IPOPT's watchdog (watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3) would change:
the compiled restatement (oracle/cpl_solve_host.c, cplo_set_watchdog) with and without it, on
TestBasic's four scenarios from x = 0 (IFOPT's limited-memory default, max_iter 3000) and on a sample
of the solve5 workload (both Hessian modes).  Per case: status, iterations, objective, and the
watchdog's events (starts, successes, restorations of the kept iterate).  CPU only.

python scripts/watchdog_effect.py [sample] > profiles/r5/watchdog_effect.json
"""
import json
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]

import pyoracle  # noqa: E402
from centroidalplanner_amd.workload import solve_inputs, solve_problem  # noqa: E402
from testbasic_outcomes import com_planner, ground, simple, superquadric  # noqa: E402

STATUS = {0: "optimal", 1: "acceptable", 2: "max_iter", 3: "local_infeasibility", 4: "restoration_failed"}


def one(desc, x0, mass, hessian, max_iter, wd):
    pyoracle.set_watchdog(wd)
    pyoracle.watchdog_events()
    r = pyoracle.solve(desc, x0, mass, max_iter=max_iter, hessian=hessian)
    ev = pyoracle.watchdog_events()
    pyoracle.set_watchdog(False)
    return {"status": STATUS[r["status"]], "iterations": r["iterations"], "objective": r["objective"],
            "restorations": r["restorations"], "wd_starts": ev[0], "wd_successes": ev[1], "wd_restores": ev[2]}


def main():
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    out = {"what": "compiled restatement without / with IPOPT's watchdog (trigger 10, trial max 3)",
           "command": "python scripts/watchdog_effect.py " + " ".join(sys.argv[1:]), "testbasic": {}, "solve5": {}}
    for name, make in (("testSimpleProblem", simple), ("testGroundEnv", ground),
                       ("testSuperquadricEnv", superquadric), ("testCoMPlanner", com_planner)):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            cpl = make()[0]
            prob = cpl.GetCplProblem()
            x0 = prob.get_starting_point()
        out["testbasic"][name] = {w: one(prob.desc(), x0, prob.desc().mass, "limited-memory", 3000, w == "on")
                                  for w in ("off", "on")}
        print(name, json.dumps(out["testbasic"][name]), file=sys.stderr, flush=True)
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, sample)
    for hessian in ("limited-memory", "exact"):
        rows = {"off": [], "on": []}
        for b in range(sample):
            for w in ("off", "on"):
                rows[w].append(one(prob.desc(), X0[b], mass[b], hessian, 3000, w == "on"))
        summ = {}
        for w, rs in rows.items():
            its = np.array([r["iterations"] for r in rs])
            summ[w] = {"statuses": {s: sum(r["status"] == s for r in rs) for s in sorted({r["status"] for r in rs})},
                       "iterations_mean": float(its.mean()), "iterations_max": int(its.max()),
                       "wd_starts": sum(r["wd_starts"] for r in rs), "wd_successes": sum(r["wd_successes"] for r in rs),
                       "wd_restores": sum(r["wd_restores"] for r in rs)}
        changed = [b for b in range(sample) if rows["off"][b]["iterations"] != rows["on"][b]["iterations"]
                   or rows["off"][b]["status"] != rows["on"][b]["status"]]
        dobj = [abs(rows["on"][b]["objective"] - rows["off"][b]["objective"]) / max(abs(rows["off"][b]["objective"]), 1e-300)
                for b in range(sample)]
        summ["instances"] = sample
        summ["instances_changed"] = len(changed)
        summ["max_rel_objective_change"] = float(max(dobj))
        summ["changed_examples"] = [{"instance": b, "off": rows["off"][b], "on": rows["on"][b]} for b in changed[:5]]
        out["solve5"][hessian] = summ
        print(hessian, json.dumps({k: v for k, v in summ.items() if k != "changed_examples"}), file=sys.stderr,
              flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
