"""How fast would a kind-partitioned mixed batch be?  Times the eval kernel on 1,048,576 mixed
16-contact instances against 524,288 all-Superquadric + 524,288 all-Ground 16-contact instances
(the two halves a stable partition by environment tag would produce), HIP events on the stream."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import generate, make_problem  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream()


def timed(env, B, reps=10):
    prob = make_problem(16, env)
    x, mass, tag = generate(16, env, B, 7)
    xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
    tt = torch.tensor(tag, device=dev) if tag is not None else None
    n, m, nnz = prob.n, prob.m, prob.nnz
    g = torch.empty(B, m, dtype=torch.float64, device=dev)
    j = torch.empty(B, nnz, dtype=torch.float64, device=dev)
    ms = ctypes.c_double()
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    _abi.check(_abi.lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(g), p(j), None,
                                            None, None, ctypes.c_void_p(s.cuda_stream), reps, ctypes.byref(ms)))
    return ms.value


mixed = timed("mixed", 1 << 20)
sq = timed("superquadric", 1 << 19)
gr = timed("ground", 1 << 19)
print(f"mixed 1M x 16: {mixed:.3f} ms; SQ 512k x 16: {sq:.3f} ms + Ground 512k x 16: {gr:.3f} ms = {sq + gr:.3f} ms")
