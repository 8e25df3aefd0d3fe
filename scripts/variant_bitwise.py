"""Eval-kernel variants (cpl_set_tuning) against the default on the same inputs: bitwise equality of g
and the Jacobian values (NaN positions included), for a mixed batch with random tags and the two
one-kind batches.  GPU box; one JSON line per (config, variant).
    python scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 6:0:256:1,0:0:256:1:1024"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs, generate  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="mixed16")
ap.add_argument("--batch", type=int, default=20011)
ap.add_argument("--variants", default="6:0:256:1")
args = ap.parse_args()
cfg = CONFIGS[args.config]
dev = torch.device("cuda:0")
p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def run(prob, xt, mt, tt, v):
    n, m, nnz = prob.get_nlp_info()
    B = xt.shape[0]
    _abi.check(_abi.lib.cpl_set_tuning(v[0], v[1], v[2], v[3], v[4] if len(v) > 4 else 0))
    g = torch.full((B, m), -7.0, dtype=torch.float64, device=dev)
    j = torch.full((B, nnz), -7.0, dtype=torch.float64, device=dev)
    _abi.check(_abi.lib.cpl_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), p(tt), p(g), p(j), None, None, None))
    torch.cuda.synchronize()
    _abi.check(_abi.lib.cpl_set_tuning(0, 0, 256, 1, 0))
    return g.cpu().numpy(), j.cpu().numpy()


def same(a, b):
    return bool(np.array_equal(a.view(np.int64), b.view(np.int64)))


prob, x, mass, tag = config_inputs(cfg, args.batch)
cases = {"random": (x, tag)}
if tag is not None:
    for kind, t in (("all_sq", 2), ("all_ground", 1)):
        xk, _, _ = generate(cfg.n_contacts, "superquadric" if t == 2 else "ground", args.batch, 4243)
        cases[kind] = (xk, np.full(args.batch, t, np.uint8))
ok_all = True
for name, (xc, tc) in cases.items():
    xt, mt = torch.tensor(xc, device=dev), torch.tensor(mass, device=dev)
    tt = None if tc is None else torch.tensor(tc, device=dev)
    ref = run(prob, xt, mt, tt, (0, 0, 256, 1, 0))
    for s in args.variants.split(","):
        v = tuple(int(q) for q in s.split(":"))
        got = run(prob, xt, mt, tt, v)
        eq = same(ref[0], got[0]) and same(ref[1], got[1])
        ok_all &= eq
        print(json.dumps({"config": args.config, "case": name, "batch": args.batch, "variant": s, "bitwise": eq}),
              flush=True)
sys.exit(0 if ok_all else 1)
