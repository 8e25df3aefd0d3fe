"""The mixed split's co-run against its streams' hardware queues: the same mixed16 launch timed on the
current stream and on several fresh streams created up front (each main stream gets its own side stream at
its first launch, so the (main, side) pairs land on different HSA queues of the process's pool,
GPU_MAX_HW_QUEUES = 4).  One JSON line per stream: median / min ms over interleaved rounds.

python scripts/mixed_stream_probe.py [--streams 6] [--rounds 5] [--reps 10] [--batch 0]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="mixed16")
ap.add_argument("--streams", type=int, default=6)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--batch", type=int, default=0)
args = ap.parse_args()

cfg = CONFIGS[args.config]
B = args.batch or cfg.batch
prob, x, mass, tag = config_inputs(cfg, B)
dev = torch.device("cuda:0")
xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
tt = None if tag is None else torch.tensor(tag, device=dev)
out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac"))
norms = torch.zeros(2, dtype=torch.float64, device=dev)
streams = [("current", torch.cuda.current_stream())] + [(f"new{i}", torch.cuda.Stream()) for i in range(args.streams)]
torch.cuda.synchronize()


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


times = {name: [] for name, _ in streams}
for _ in range(args.rounds):
    for name, s in streams:
        ms = ctypes.c_double()
        _abi.check(_abi.lib.cpl_time_eval_batch_ex(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(out["g"]),
                                                   p(out["jac"]), None, None, p(norms), 0,
                                                   ctypes.c_void_p(s.cuda_stream), args.reps, ctypes.byref(ms)))
        times[name].append(ms.value)
for name, ts in times.items():
    print(json.dumps({"config": args.config, "batch": B, "stream": name, "median_ms": statistics.median(ts),
                      "min_ms": min(ts), "max_ms": max(ts)}), flush=True)
