"""A/B of two builds of the HIP library in ONE process (interleaved rounds, same inputs/outputs).

python scripts/ab_libs.py --config sq8 --libs centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_old.so
Both libraries export the same C-ABI; each is loaded under its own handle (RTLD_LOCAL) and timed with
its own cpl_time_eval_batch (HIP events on the launch stream).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench import algorithmic_bytes  # noqa: E402
from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="sq8")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--libs", default="centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_old.so")
ap.add_argument("--tuning", default="", help="variant:lds_kb:wg:nt passed to every library's cpl_set_tuning")
ap.add_argument("--no-norms", action="store_true", help="time the eval kernel without the fused residual norms")
ap.add_argument("--tags", default="", help="mixed configs: all_sq | all_ground (every instance of one kind)")
args = ap.parse_args()

libs = {}
for tag in args.libs.split(","):
    path = tag
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in ("cpl_time_eval_batch", "cpl_eval_batch"):
        fn = getattr(lib, name)
        res, sig = _abi.SIGNATURES[name]
        fn.restype, fn.argtypes = res, sig
    if args.tuning:
        v = [int(t) for t in args.tuning.split(":")]
        lib.cpl_set_tuning.restype = ctypes.c_int32
        _abi.check(lib.cpl_set_tuning(*[ctypes.c_int32(t) for t in (v + [0] * (5 - len(v)))]))
    libs[tag] = lib

cfg = CONFIGS[args.config]
B = args.batch or cfg.batch
prob, x, mass, tag = config_inputs(cfg, B)
if args.tags:  # one kind only, through the mixed launch (the kind split's halves alone)
    import numpy as np

    from centroidalplanner_amd.workload import generate

    kind = "superquadric" if args.tags == "all_sq" else "ground"
    x, _, _ = generate(cfg.n_contacts, kind, B, 4242)
    tag = np.full(B, 2 if kind == "superquadric" else 1, np.uint8)
dev = torch.device("cuda:0")
xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
tt = None if tag is None else torch.tensor(tag, device=dev)
out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
stream = torch.cuda.current_stream()
p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
times = {k: [] for k in libs}
# the libraries' order alternates per round: with a fixed order the second library measured ~2-3 %
# faster on sq8 even when both were the same build (profiles/r5/sq_prio/order/same)
for rnd in range(args.rounds):
    for k, lib in (list(libs.items()) if rnd % 2 == 0 else list(libs.items())[::-1]):
        ms = ctypes.c_double()
        _abi.check(lib.cpl_time_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(out["g"]), p(out["jac"]),
                                           None, None, None if args.no_norms else p(out["norms"]),
                                           ctypes.c_void_p(stream.cuda_stream), args.reps,
                                           ctypes.byref(ms)))
        times[k].append(ms.value)
# every library's outputs on the same inputs, compared bit for bit with the first one's
ref = None
for k, lib in libs.items():
    g, jac = torch.full_like(out["g"], float("nan")), torch.full_like(out["jac"], float("nan"))
    _abi.check(lib.cpl_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(g), p(jac), None, None,
                                  ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
    if ref is None:
        ref = (k, g, jac)
    else:
        same = all(bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all()) for a, b in ((g, ref[1]), (jac, ref[2])))
        print(json.dumps({"lib": k, "bitwise_equal_to": ref[0], "equal": same}), flush=True)
bpi, m = algorithmic_bytes(cfg.n_contacts, cfg.env)
for k, ts in times.items():
    med = statistics.median(ts)
    print(json.dumps({"config": args.config, "batch": B, "lib": k, "tuning": args.tuning, "norms": not args.no_norms,
                      "median_ms": med, "min_ms": min(ts),
                      "GBps": bpi * B / (med * 1e-3) / 1e9}), flush=True)
