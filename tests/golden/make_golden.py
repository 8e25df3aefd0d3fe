"""Generates the golden fixtures in tests/golden/*.npz from the oracle (CPU restatement).

The reference itself cannot be built here (no Eigen / IFOPT / IPOPT) and its tests hold no golden
vectors, so these fixtures pin the oracle as it stands (after its solve-level pinning by the
TestBasic scenarios, tests/test_oracle_pinning.py) and let the GPU path be checked against stored
data.  Every fixture: seeded inputs (x, mass, env tag) + every output (g, jac, f, grad) + the
problem template parameters.  Regenerate with:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402
from centroidalplanner_amd.workload import generate, make_problem  # noqa: E402

CASES = [
    # name, N, env, B, F_thr, stress
    ("ground_n1", 1, "ground", 16, 0.0, False),
    ("ground_n4", 4, "ground", 16, 0.0, False),
    ("ground_n4_thr20", 4, "ground", 16, 20.0, False),
    ("none_n4_thr20", 4, "none", 16, 20.0, False),
    ("sq_n4", 4, "superquadric", 16, 0.0, False),
    ("sq_n8", 8, "superquadric", 16, 0.0, False),
    ("sq_n8_stress", 8, "superquadric", 16, 0.0, True),
    ("ground_n12", 12, "ground", 8, 0.0, False),
    ("mixed_n16", 16, "mixed", 8, 0.0, False),
    ("none_n3", 3, "none", 16, 0.0, False),
]


def build(name, N, env, B, thr, stress):
    prob = make_problem(N, env)
    for c in prob.contact_names:
        prob.SetForceThreshold(c, thr)
    x, mass, tag = generate(N, env, B, sum(map(ord, name)), stress=stress)  # seed: stable per case name
    if name.startswith("ground_n4"):
        x[0] = 0.0            # the IPOPT start point (NaN cone Jacobians)
    out = pyoracle.eval_batch(prob.desc(), x, mass, tag, nthreads=1)
    return dict(x=x, mass=mass, tag=np.zeros(B, np.uint8) if tag is None else tag, N=N, env=env, F_thr=thr, **out)


if __name__ == "__main__":
    for case in CASES:
        d = build(*case)
        np.savez_compressed(os.path.join(HERE, case[0] + ".npz"), **d)
        print(case[0], {k: getattr(v, "shape", v) for k, v in d.items()})
