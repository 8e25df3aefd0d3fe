"""Raw HBM ceilings of this MI355X for context, HIP-event timed, one JSON line:
write-only (fill), copy (1 read : 1 write) and read-only (sum) on 2 GiB buffers, plus the eval
kernel's own traffic shape — 1 read : 5 writes ("expand5": each double read is written 5 times,
320 B in : 1632 B out per Ground instance) — at the bench's 128 MB working set (65,536 x 4
instances, inside the 256 MiB Infinity Cache) and at 2 GiB (the 1,048,576 x 4 north star)."""
import json

import torch

dev = torch.device("cuda:0")


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


res = {}
n = (2 << 30) // 8
a = torch.empty(n, dtype=torch.float64, device=dev)
b = torch.empty(n, dtype=torch.float64, device=dev)
a.fill_(1.0)
nbytes = n * 8
res["write_GBps"] = nbytes / t(lambda: b.fill_(2.0)) / 1e9
res["copy_GBps"] = 2 * nbytes / t(lambda: b.copy_(a)) / 1e9
res["read_GBps"] = nbytes / t(lambda: a.sum()) / 1e9
for label, total in (("expand5_128MB_GBps", 128 << 20), ("expand5_2GiB_GBps", 2 << 30)):
    nr = total // 8 // 6
    src = a[:nr].view(-1, 1)
    dst = b[:5 * nr].view(-1, 5)
    res[label] = 6 * nr * 8 / t(lambda: dst.copy_(src.expand(-1, 5))) / 1e9
print(json.dumps(res))
