"""cpl_kkt_solve (csrc/cpl_kkt.hip): the solve loop's batched Newton step on the GPU, against a dense
numpy solve of the same KKT systems (float64; tolerance 1e-9 relative to the solution's scale, the
systems' condition numbers are ~1e3-1e5).

The 4-contact size (nw 47, m 30) runs the one-wave kernel from 64 systems up and the workgroup kernel
below (every other size: the workgroup kernel's generic instance): the (47, 30) cases run at B = 64 /
300 and B = 4,096 (the dense check on a sample of the large batches), the small-batch cases and
the other sizes cover the workgroup kernel."""
import ctypes

import numpy as np
import pytest

from centroidalplanner_amd import _abi


def test_workspace_size_and_argument_checks():
    nw, m = 47, 30
    nz = nw - m
    assert _abi.lib.cpl_kkt_workspace_doubles(nw, m) == nw * nw + m * nw + nz * nz + 4
    assert _abi.lib.cpl_kkt_workspace_doubles(10, 11) == -1
    # m > nw and nw > 128 are rejected before any device work
    st = _abi.lib.cpl_kkt_solve(0, 1, 10, 11, *([None] * 13), None)
    assert st == _abi.ERR_INVALID_ARGUMENT
    st = _abi.lib.cpl_kkt_solve(0, 1, 200, 10, *([None] * 13), None)
    assert st == _abi.ERR_INVALID_ARGUMENT


def _systems(B, nw, m, seed, indefinite=False, rank_def=False):
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(B, m, nw))
    if rank_def:
        A[:, -1] = A[:, 0] + A[:, 1]  # a redundant constraint row
    X = rng.normal(size=(B, nw, nw))
    M = X @ X.transpose(0, 2, 1) / nw + np.eye(nw) * 0.1
    if indefinite:
        M -= 3.0 * np.eye(nw)  # negative curvature also on null(A)
    r1 = rng.normal(size=(B, nw))
    r2 = rng.normal(size=(B, m))
    return M, A, r1, r2


def _run(mode, M, A, r1, r2, mu, ws=None, last=None):
    import torch

    dev = torch.device("cuda:0")
    B, m, nw = A.shape
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Mt, At, r1t, r2t, mut = T(M), T(A), T(r1), T(r2), T(mu)
    lastt = T(last if last is not None else np.zeros(B))
    dw = torch.empty(B, nw, dtype=torch.float64, device=dev)
    dy = torch.empty(B, m, dtype=torch.float64, device=dev)
    dW = torch.empty(B, dtype=torch.float64, device=dev)
    dC = torch.empty(B, dtype=torch.float64, device=dev)
    info = torch.empty(B, dtype=torch.int32, device=dev)
    if ws is None:
        ws = torch.empty(B * _abi.lib.cpl_kkt_workspace_doubles(nw, m), dtype=torch.float64, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _abi.check(_abi.lib.cpl_kkt_solve(mode, B, nw, m, p(Mt), p(At), p(r1t), p(r2t), p(mut), p(lastt), None, p(dw),
                                      p(dy), p(dW), p(dC), p(info), p(ws), None))
    torch.cuda.synchronize()
    return dw.cpu().numpy(), dy.cpu().numpy(), dW.cpu().numpy(), dC.cpu().numpy(), info.cpu().numpy(), ws


def _dense(M, A, r1, r2, dW=None):
    B, m, nw = A.shape
    out = []
    for b in range(B):
        K = np.zeros((nw + m, nw + m))
        K[:nw, :nw] = M[b] + (0.0 if dW is None else dW[b]) * np.eye(nw)
        K[:nw, nw:] = A[b].T
        K[nw:, :nw] = A[b]
        out.append(np.linalg.solve(K, np.concatenate([r1[b], r2[b]])))
    out = np.array(out)
    return out[:, :nw], out[:, nw:]


def _sample(B):
    return np.unique(np.concatenate([np.arange(min(B, 200)), np.arange(max(B - 100, 0), B)]))


@pytest.mark.gpu
@pytest.mark.parametrize("nw,m,B", [(47, 30, 16), (47, 30, 300), (47, 30, 4096), (39, 14, 300), (12, 12, 300), (20, 0, 300),
                                    (91, 54, 300), (100, 70, 300)])
def test_kkt_matches_dense_solve(nw, m, B):
    nz = nw - m
    if 8 * (nw * nw + m * nw + nz * nz + nw + m + max(2 * nw, 3 * m) + 8) > 160 * 1024:
        pytest.skip("LDS image above 160 KiB: rejected by design")
    M, A, r1, r2 = _systems(B, nw, m, seed=nw + m)
    dw, dy, dW, dC, info, _ = _run(0, M, A, r1, r2, np.full(B, 0.1))
    assert (info == 0).all() and (dW == 0).all() and (dC == 0).all()
    idx = _sample(B)
    M, A, r1, r2, dw, dy = M[idx], A[idx], r1[idx], r2[idx], dw[idx], dy[idx]
    rw, ry = _dense(M, A, r1, r2)
    np.testing.assert_allclose(dw, rw, rtol=0, atol=1e-9 * np.abs(rw).max())
    if m:
        np.testing.assert_allclose(dy, ry, rtol=0, atol=1e-9 * np.abs(ry).max())


@pytest.mark.gpu
@pytest.mark.parametrize("B", [64, 4096])
def test_kkt_inertia_correction_and_resolve(B):
    nw, m = 47, 30
    M, A, r1, r2 = _systems(B, nw, m, seed=3, indefinite=True)
    dw, dy, dW, dC, info, ws = _run(0, M, A, r1, r2, np.full(B, 0.1))
    assert (info == 0).all() and (dW > 0).all()
    idx = _sample(B)
    # the returned step solves the system with delta_w added (IPOPT's corrected system)
    rw, ry = _dense(M[idx], A[idx], r1[idx], r2[idx], dW[idx])
    np.testing.assert_allclose(dw[idx], rw, rtol=0, atol=1e-8 * np.abs(rw).max())
    # and the reduced Hessian of the corrected system is positive definite
    for b in range(4):
        q, _ = np.linalg.qr(A[b].T, mode="complete")
        Z = q[:, m:]
        assert np.linalg.eigvalsh(Z.T @ (M[b] + dW[b] * np.eye(nw)) @ Z).min() > 0
    # mode 1: another r2 with the kept factors == a dense solve of the corrected system
    r2b = np.random.default_rng(9).normal(size=(B, m))
    dw1, dy1, *_ = _run(1, M, A, r1, r2b, np.full(B, 0.1), ws=ws)
    rw1, _ = _dense(M[idx], A[idx], r1[idx], r2b[idx], dW[idx])
    np.testing.assert_allclose(dw1[idx], rw1, rtol=0, atol=1e-7 * np.abs(rw1).max())


@pytest.mark.gpu
@pytest.mark.parametrize("B", [32, 4096])
def test_kkt_rank_deficient_gets_delta_c(B):
    nw, m = 47, 30
    M, A, r1, r2 = _systems(B, nw, m, seed=4, rank_def=True)
    r2[:, -1] = r2[:, 0] + r2[:, 1]  # consistent right-hand side
    dw, dy, dW, dC, info, _ = _run(0, M, A, r1, r2, np.full(B, 1e-2))
    assert (dC > 0).all() and np.isfinite(dw).all() and np.isfinite(dy).all()
    # the primal step still satisfies the (consistent) linearised constraints
    np.testing.assert_allclose(np.einsum("bmn,bn->bm", A, dw), r2, atol=1e-6)
