"""The single-instance TNLP callback path (cpl_eval_batch_host, B = 1 and a few small batches) under
each eval kernel variant (cpl_set_tuning): which kernel has the shortest launch-to-completion latency
for a handful of instances.  Interleaved rounds, median us per call; the outputs' bits per variant
checked against the default's.   python scripts/hostio_variants.py [--config ground4] [--reps 400]"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="ground4")
ap.add_argument("--reps", type=int, default=400)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--batches", default="1,4,32")
ap.add_argument("--variants", default="0,1,2,3,5")
args = ap.parse_args()
cfg = CONFIGS[args.config]
prob = config_inputs(cfg, batch=1)[0]
desc = prob.desc()
n, m, nnz = prob.get_nlp_info()
ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
for B in [int(b) for b in args.batches.split(",")]:
    _, x, mass, tag = config_inputs(cfg, batch=B)
    x = np.ascontiguousarray(x, dtype=np.float64)
    tag = None if tag is None else np.ascontiguousarray(tag, dtype=np.uint8)
    outs = {}
    times = {v: [] for v in args.variants.split(",")}
    for _ in range(args.rounds):
        for v in times:
            _abi.check(_abi.lib.cpl_set_tuning(int(v), 0, 256, 1, 0))
            g, j = np.empty((B, m)), np.empty((B, nnz))
            for _ in range(20):
                _abi.check(_abi.lib.cpl_eval_batch_host(ctypes.byref(desc), B, ptr(x), ptr(mass), ptr(tag), ptr(g), ptr(j),
                                                        None, None, None, 0))
            t0 = time.perf_counter()
            for _ in range(args.reps):
                _abi.lib.cpl_eval_batch_host(ctypes.byref(desc), B, ptr(x), ptr(mass), ptr(tag), ptr(g), ptr(j), None, None,
                                             None, 0)
            times[v].append((time.perf_counter() - t0) / args.reps * 1e6)
            outs[v] = (g.copy(), j.copy())
    _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    g0, j0 = outs["0"]
    for v, ts in times.items():
        g, j = outs[v]
        print(json.dumps({"config": args.config, "batch": B, "variant": int(v), "us_median": statistics.median(ts),
                          "us_min": min(ts), "bitwise_default": bool(np.array_equal(g, g0, equal_nan=True)
                                                                    and np.array_equal(j, j0, equal_nan=True))}),
              flush=True)
