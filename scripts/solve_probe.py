"""Timing probe of the batched solve loop's linear-algebra building blocks on the GPU (prints as it goes)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
dev = torch.device("cuda:0")
dt = torch.float64
for B in (512, 2048, 8192):
    A = torch.randn(B, 30, 47, dtype=dt, device=dev)
    Mz = torch.randn(B, 17, 17, dtype=dt, device=dev); Mz = Mz @ Mz.transpose(1, 2) + torch.eye(17, dtype=dt, device=dev)
    def t(f, name, reps=3):
        f(); torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(reps): f()
        torch.cuda.synchronize(); print(f"B={B} {name}: {(time.perf_counter()-t0)/reps*1e3:.2f} ms", flush=True)
    t(lambda: torch.linalg.qr(A.transpose(1, 2), mode="complete"), "qr complete 47x30")
    t(lambda: torch.linalg.cholesky_ex(Mz), "cholesky_ex 17x17")
    L = torch.linalg.cholesky(Mz)
    rhs = torch.randn(B, 17, 1, dtype=dt, device=dev)
    t(lambda: torch.cholesky_solve(rhs, L), "cholesky_solve 17")
    R = torch.triu(torch.randn(B, 30, 30, dtype=dt, device=dev)) + 10 * torch.eye(30, dtype=dt, device=dev)
    r = torch.randn(B, 30, 1, dtype=dt, device=dev)
    t(lambda: torch.linalg.solve_triangular(R, r, upper=True), "solve_triangular 30")
    t(lambda: A @ A.transpose(1, 2), "bmm 30x47x30")
