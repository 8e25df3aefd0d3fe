"""Raw HBM ceilings of this MI355X for context: write-only (fill), copy (1 read : 1 write) and
read-only (sum) on 2 GiB buffers, HIP-event timed.  Prints one JSON line."""
import json

import torch

dev = torch.device("cuda:0")
n = (2 << 30) // 8
a = torch.empty(n, dtype=torch.float64, device=dev)
b = torch.empty(n, dtype=torch.float64, device=dev)
a.fill_(1.0)


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


nbytes = n * 8
res = {
    "write_GBps": nbytes / t(lambda: b.fill_(2.0)) / 1e9,
    "copy_GBps": 2 * nbytes / t(lambda: b.copy_(a)) / 1e9,
    "read_GBps": nbytes / t(lambda: a.sum()) / 1e9,
}
print(json.dumps(res))
