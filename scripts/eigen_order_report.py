"""Per-class deviation between the two plausible Eigen reduction orders of the reference (SSE2
packets vs no packet math for a 3-vector), with histograms, on the parity input sets and on the
same inputs moved onto the friction-cone boundary (tests/eigen_order.py).  CPU only.
    python scripts/eigen_order_report.py profiles/r5/eigen_order_hist.json [batch]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from eigen_order import cone_active, histogram, order_deviation  # noqa: E402
from centroidalplanner_amd.workload import generate, make_problem  # noqa: E402

out_path = sys.argv[1] if len(sys.argv) > 1 else "eigen_order_hist.json"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
report = {"what": "oracle (SSE2 order (a0b0 + a1b1) + a2b2) against the oracle built with -DCPLO_EIGEN_REDUX_NOVEC "
                  "(a0b0 + (a1b1 + a2b2)); same inputs; per output class",
          "command": "python scripts/eigen_order_report.py " + " ".join(sys.argv[1:]),
          "batch": B, "cases": {}}
for N, env in ((4, "ground"), (8, "superquadric"), (16, "mixed"), (4, "none")):
    prob = make_problem(N, env)
    x, mass, tag = generate(N, env, B, 9000 + N)
    for label, xx in (("interior", x), ("cone_active", cone_active(x, N, prob.GetMu()))):
        key = f"{env}_n{N}_{label}"
        report["cases"][key] = {"deviation": order_deviation(prob, env, xx, mass, tag),
                                "histogram": histogram(prob, env, xx, mass, tag)}
        print(key, {k: (v["differ"], v["max_rel"], v.get("max_rel_uncancelled")) for k, v in
                    report["cases"][key]["deviation"].items() if isinstance(v, dict) and v["differ"]}, flush=True)
worst = {}
for case in report["cases"].values():
    for k, v in case["deviation"].items():
        if isinstance(v, dict):
            w = worst.setdefault(k, {"max_rel": 0.0, "max_rel_uncancelled": 0.0, "max_abs": 0.0})
            for f in w:
                if f in v:
                    w[f] = max(w[f], v[f])
report["worst_per_class"] = worst
with open(out_path, "w") as fh:
    json.dump(report, fh, indent=1, default=str)
print(json.dumps(worst, indent=1, default=str))
