"""The shard evaluation of bench.py's CPU rehearsal (--rehearse-cpu, tests only): the oracle stands in
for the rank's GPU and returns the shard's residual norms [max violation, sum of squared violations]
against the constraint bounds (what cpl_eval_batch_norms computes on the device)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


def norms(prob, x, mass, tag):
    import pyoracle

    fail = os.environ.get("CPL_REHEARSAL_FAIL_RANK")
    if fail is not None and fail == os.environ.get("RANK"):
        raise RuntimeError("rehearsal: this rank fails on purpose")
    g = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=("g",), nthreads=1)["g"]
    _, _, gl, gu = prob.get_bounds_info()
    viol = np.maximum(np.maximum(gl - g, g - gu), 0.0)
    viol = np.where(np.isnan(g), np.inf, viol)
    return [float(viol.max(initial=0.0)), float((viol ** 2).sum())]
