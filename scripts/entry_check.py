"""Entry kernel (variant 5) against the pipelined kernel (variant 2) at 1,048,576 x 4 Ground, for each
library given: which instances differ (diagnostic)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from centroidalplanner_amd import _abi
from centroidalplanner_amd.workload import generate, make_problem
prob = make_problem(4, "ground")
x, mass, _ = generate(4, "ground", 1 << 20, 5)
dev = torch.device("cuda:0")
xt, mt = torch.tensor(x, device=dev), torch.tensor(mass, device=dev)
n, m, nnz = prob.get_nlp_info()
B = x.shape[0]
p = lambda t: ctypes.c_void_p(t.data_ptr())
for path in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in ("cpl_eval_batch", "cpl_set_tuning"):
        fn = getattr(lib, name); res, sig = _abi.SIGNATURES[name]; fn.restype, fn.argtypes = res, sig
    outs = {}
    for v in (2, 5):
        _abi.check(lib.cpl_set_tuning(v, 0, 256, 1, 0))
        g = torch.full((B, m), float("nan"), dtype=torch.float64, device=dev)
        j = torch.full((B, nnz), float("nan"), dtype=torch.float64, device=dev)
        _abi.check(lib.cpl_eval_batch(ctypes.byref(prob.desc()), B, p(xt), p(mt), None, p(g), p(j), None, None, None))
        torch.cuda.synchronize()
        outs[v] = (g, j)
    _abi.check(lib.cpl_set_tuning(0, 0, 256, 1, 0))
    bad = ((outs[2][0] != outs[5][0]) & ~(torch.isnan(outs[2][0]) & torch.isnan(outs[5][0]))).any(1)
    idx = torch.nonzero(bad).flatten()
    print(path, "differing instances:", idx.numel(), idx[:5].tolist(), idx[-5:].tolist() if idx.numel() else [],
          "nan in entry g:", int(torch.isnan(outs[5][0]).any(1).sum()), flush=True)
