"""Launches one eval configuration a few times under a given tuning variant (for rocprofv3 kernel traces).

python scripts/prof_eval.py <config> <variant> [lds_kb] [reps]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from centroidalplanner_amd import _abi  # noqa: E402
from centroidalplanner_amd.workload import CONFIGS, config_inputs  # noqa: E402

cfg = CONFIGS[sys.argv[1]]
variant = int(sys.argv[2])
lds = int(sys.argv[3]) if len(sys.argv) > 3 else 0
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
prob, x, mass, tag = config_inputs(cfg)
dev = torch.device("cuda:0")
xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
tt = None if tag is None else torch.tensor(tag, device=dev)
_abi.check(_abi.lib.cpl_set_tuning(variant, lds, 256, 1, 0))
out = prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"))
for _ in range(reps):
    prob.eval_batch(xt, mt, tt, outputs=("g", "jac", "norms"), out=out)
torch.cuda.synchronize()
print("done", cfg.name, variant, lds)
