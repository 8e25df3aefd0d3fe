"""Latency of the host-array entry point (cpl_eval_batch_host) at small batches: the single-instance
TNLP callback path and where batching starts to pay.  Host arrays are ordinary numpy (pageable)
memory, as IPOPT hands them over.

python scripts/hostio_latency.py [--config ground4_1m] [--reps 2000]

"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="ground4_1m")
ap.add_argument("--reps", type=int, default=2000)
ap.add_argument("--batches", default="1,4,16,64,256,1024,4096")
args = ap.parse_args()

cfg = CONFIGS[args.config]
prob = config_inputs(cfg, batch=1)[0]
desc = prob.desc()
n, m, nnz = prob.get_nlp_info()
ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
out = {"config": args.config, "us": {}}
for B in [int(b) for b in args.batches.split(",")]:
    _, x, mass, tag = config_inputs(cfg, batch=B)
    x = np.ascontiguousarray(x, dtype=np.float64)
    tag = None if tag is None else np.ascontiguousarray(tag, dtype=np.uint8)
    g, j = np.empty((B, m)), np.empty((B, nnz))

    def once():
        _abi.check(_abi.lib.cpl_eval_batch_host(ctypes.byref(desc), B, ptr(x), None, ptr(tag), ptr(g), ptr(j),
                                                None, None, None, 0))

    reps = max(20, args.reps // max(1, B // 16))
    for _ in range(20):
        once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    out["us"][B] = (time.perf_counter() - t0) / reps * 1e6
print(json.dumps(out), flush=True)
