"""Correctness probe of torch's batched dense linear algebra on the GPU vs CPU (small batch)."""
import torch
dt = torch.float64
dev = torch.device("cuda:0")
torch.manual_seed(0)
for B, n, k in ((4, 17, 1), (512, 30, 47), (512, 47, 1), (512, 47, 3)):
    X = torch.randn(B, n, n, dtype=dt)
    S = X @ X.transpose(1, 2) + n * torch.eye(n, dtype=dt)
    R = torch.randn(B, n, k, dtype=dt)
    Lc, ic = torch.linalg.cholesky_ex(S)
    Lg, ig = torch.linalg.cholesky_ex(S.to(dev))
    xc = torch.cholesky_solve(R, Lc)
    xg = torch.cholesky_solve(R.to(dev), Lg).cpu()
    print(f"B={B} n={n} nrhs={k}: chol max|dL|={float((Lg.cpu() - Lc).abs().max()):.2e} info_gpu_nonzero={int((ig != 0).sum())} "
          f"solve max|dx|={float((xg - xc).abs().max()):.2e} |x|={float(xc.abs().max()):.2e}", flush=True)
    # indefinite: info must be nonzero
    Si = S - 3 * n * torch.eye(n, dtype=dt)
    _, ic2 = torch.linalg.cholesky_ex(Si)
    _, ig2 = torch.linalg.cholesky_ex(Si.to(dev))
    print(f"   indefinite: info cpu nonzero {int((ic2 != 0).sum())} gpu nonzero {int((ig2 != 0).sum())} (of {B})", flush=True)
