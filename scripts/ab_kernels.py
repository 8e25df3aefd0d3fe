"""A/B of eval-kernel variants in ONE process, interleaved rounds (guide §5.4 rule 24).

python scripts/ab_kernels.py [--config ground4] [--rounds 5] [--reps 20]
Prints one JSON line per (variant, lds budget) with median / min ms and achieved GB/s.
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
ap.add_argument("--config", default="ground4")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--variants", default="0:0:256:1,3:32:256:1,2:48:256:1")
ap.add_argument("--outputs", default="g,jac")
ap.add_argument("--norms", action="store_true", help="fused residual norms (cpl_eval_batch_norms)")
ap.add_argument("--folded", action="store_true", help="values-only Jacobian records (CPL_EVAL_JAC_FOLDED)")
ap.add_argument("--soa", action="store_true", help="entry-major outputs (CPL_EVAL_SOA)")
ap.add_argument("--tags", default="", help="mixed configs: all_sq | all_ground (every instance of one kind)")
args = ap.parse_args()

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
outs = tuple(args.outputs.split(","))
out = prob.eval_batch(xt, mt, tt, outputs=outs, jac_folded=args.folded, soa=args.soa)
flags = (_abi.EVAL_JAC_FOLDED if args.folded else 0) | (_abi.EVAL_SOA if args.soa else 0)
stream = torch.cuda.current_stream()
norms = torch.zeros(2, dtype=torch.float64, device=xt.device) if args.norms else None
variants = [tuple(int(v) for v in s.split(":")) for s in args.variants.split(",")]
times = {v: [] for v in variants}


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


for _ in range(args.rounds):
    for v in variants:
        _abi.check(_abi.lib.cpl_set_tuning(v[0], v[1], v[2], v[3], v[4] if len(v) > 4 else 0))
        ms = ctypes.c_double()
        _abi.check(_abi.lib.cpl_time_eval_batch_ex(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(out.get("g")),
                                                   p(out.get("jac")), p(out.get("f")), p(out.get("grad")), p(norms),
                                                   flags, ctypes.c_void_p(stream.cuda_stream), args.reps,
                                                   ctypes.byref(ms)))
        times[v].append(ms.value)
bpi, m = algorithmic_bytes(cfg.n_contacts, cfg.env, outs)
if args.folded and "jac" in outs:
    bpi -= 8 * (prob.nnz - out["jac"].shape[1 if not args.soa else 0])
for v, ts in times.items():
    med = statistics.median(ts)
    print(json.dumps({"config": args.config, "batch": B, "folded": args.folded, "soa": args.soa, "variant": v[0], "lds_kb": v[1], "wg": v[2], "nt": v[3], "ablate": v[4] if len(v) > 4 else 0, "median_ms": med,
                      "min_ms": min(ts), "GBps": bpi * B / (med * 1e-3) / 1e9,
                      "rows_per_s": B * m / (med * 1e-3)}), flush=True)
