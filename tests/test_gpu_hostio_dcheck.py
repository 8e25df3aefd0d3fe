"""Host-buffer entry point and the batched derivative checker, on the GPU.

* cpl_eval_batch_host: numpy in / numpy out through the library's device
  workspace must equal cpl_eval_batch on device tensors bit for bit, in every layout.
* cpl_derivative_test: IPOPT's first-order derivative checker (derivative_test = "first-order",
  set by src/CentroidalPlanner.cpp:26 [IPOPT-ext]) restated below in numpy over the ORACLE's
  callbacks (forward differences of g and f, h_j = perturbation * max(1, |x_j|), an entry flagged
  when |approx - exact| / max(|approx|, tol) > tol).  IPOPT itself is absent here, so the checker's
  own semantics are "parity unpinned" against IPOPT; the GPU report must equal this restatement.
"""
import numpy as np
import pytest

import pyoracle

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _inputs(name, batch):
    from centroidalplanner_amd.workload import CONFIGS, config_inputs

    return config_inputs(CONFIGS[name], batch=batch)


def derivative_test_ref(prob, x, mass, tag, pert, tol):
    """numpy restatement: per-instance flagged counts, and the worst entry (first on ties)."""
    B, n = x.shape
    m = prob.m
    iRow, jCol = prob.get_structure()[:2]
    amap = -np.ones((m, n), dtype=np.int64)
    amap[iRow, jCol] = np.arange(len(iRow))
    base = pyoracle.eval_batch(prob.desc(), x, mass, tag, outputs=("g", "jac", "f", "grad"))
    h = pert * np.maximum(1.0, np.abs(x))                                # [B, n]
    xp = np.repeat(x[:, None, :], n, axis=1)                             # [B, n, n]
    idx = np.arange(n)
    xp[:, idx, idx] = x + h
    rep = lambda a: None if a is None else np.repeat(a, n)  # noqa: E731
    pt = pyoracle.eval_batch(prob.desc(), xp.reshape(B * n, n), rep(mass), rep(tag), outputs=("g", "f"))
    gp = pt["g"].reshape(B, n, m)
    fp = pt["f"].reshape(B, n)
    approx_f = (fp - base["f"][:, None]) / h                             # [B, n]
    approx_g = (gp - base["g"][:, None, :]) / h[:, :, None]              # [B, n, m]
    jac = base["jac"]
    exact_g = np.where(amap.T[None] >= 0, jac[:, np.maximum(amap.T, 0)], 0.0)  # [B, n, m]
    approx = np.concatenate([approx_f[:, :, None], approx_g], axis=2)   # row -1 first, then 0..m-1
    exact = np.concatenate([base["grad"][:, :, None], exact_g], axis=2)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(approx - exact) / np.maximum(np.abs(approx), tol)
    flagged = ~(rel <= tol)
    return flagged.reshape(B, -1).sum(axis=1), rel, approx, exact


# batches whose inputs + outputs fit 1 MiB take the zero-copy path (pinned staging read / written by the
# kernel), larger ones the device workspace with DMA copies; both must equal the device-array call
@pytest.mark.parametrize("name,batch,folded", [("ground4_1m", 1000, False), ("ground4_1m", 333, True),
                                               ("sq8", 64, False), ("mixed16", 40, True),
                                               ("ground4_1m", 1, False), ("ground4_1m", 1, True), ("sq8", 1, False),
                                               ("mixed16", 1, False), ("sq8", 600, True), ("mixed16", 301, False)])
def test_eval_batch_host_matches_device(name, batch, folded):
    prob, x, mass, tag = _inputs(name, batch)
    dev = torch.device("cuda:0")
    tt = torch.tensor(tag, device=dev) if tag is not None else None
    want = prob.eval_batch(torch.tensor(x, device=dev), torch.tensor(mass, device=dev), tt,
                           outputs=("g", "jac", "f", "grad", "norms"), jac_folded=folded)
    torch.cuda.synchronize()
    got = prob.eval_batch_host(x, mass, tag, outputs=("g", "jac", "f", "grad", "norms"), jac_folded=folded)
    for k in ("g", "jac", "f", "grad", "norms"):
        w = want[k].cpu().numpy()
        assert got[k].shape == w.shape, k
        assert np.array_equal(got[k].view(np.uint64), w.view(np.uint64)), k


def test_single_instance_callbacks_use_host_entry():
    prob, x, mass, _ = _inputs("ground4_1m", 1)
    prob.SetVariables(x[0])
    g = prob.eval_g(x[0])
    ref = pyoracle.eval_batch(prob.desc(), x[:1], None, outputs=("g",))["g"][0]
    assert np.array_equal(g, ref)


@pytest.mark.parametrize("pert", [1e-8, 1e-1])
def test_derivative_test_ground_matches_restatement(pert):
    prob, x, mass, _ = _inputs("ground4_1m", 300)
    dev = torch.device("cuda:0")
    tol = 1e-4
    got = prob.derivative_test(torch.tensor(x, device=dev), torch.tensor(mass, device=dev), perturbation=pert,
                               tol=tol, per_instance=True)
    cnt, rel, approx, exact = derivative_test_ref(prob, x, mass, None, pert, tol)
    B, n = x.shape
    assert got["n_checked"] == B * n * (prob.m + 1)
    assert np.array_equal(got["flagged"].cpu().numpy(), cnt)
    assert got["n_flagged"] == int(cnt.sum())
    flat = rel.reshape(-1)
    w = int(np.argmax(flat))
    b, j, r = np.unravel_index(w, rel.shape)
    assert got["max_rel_error"] == flat[w]
    assert (got["worst_instance"], got["worst_col"], got["worst_row"]) == (b, j, r - 1)
    assert got["worst_exact"] == exact[b, j, r] and got["worst_approx"] == approx[b, j, r]
    if pert == 1e-1:
        assert got["n_flagged"] > 0  # second-order terms of the cone / torque rows show at h = 0.1


def test_derivative_test_chunked_batch():
    """Past one workspace chunk (~20k instances at N=4): per-instance counts over all chunks."""
    prob, x, mass, _ = _inputs("ground4_1m", 24_000)
    dev = torch.device("cuda:0")
    got = prob.derivative_test(torch.tensor(x, device=dev), torch.tensor(mass, device=dev), per_instance=True)
    cnt, rel, _, _ = derivative_test_ref(prob, x, mass, None, 1e-8, 1e-4)
    assert np.array_equal(got["flagged"].cpu().numpy(), cnt)
    assert got["max_rel_error"] == rel.max()


@pytest.mark.parametrize("name,batch", [("sq8", 48), ("mixed16", 24)])
def test_derivative_test_superquadric(name, batch):
    """Superquadric g agrees with the oracle to ~1e-15 relative (not bitwise), and forward differences
    amplify that by 1/h: flags can only differ for entries whose deviation sits at the threshold."""
    prob, x, mass, tag = _inputs(name, batch)
    dev = torch.device("cuda:0")
    tt = torch.tensor(tag, device=dev) if tag is not None else None
    got = prob.derivative_test(torch.tensor(x, device=dev), torch.tensor(mass, device=dev), tt, per_instance=True)
    cnt, rel, _, _ = derivative_test_ref(prob, x, mass, tag, 1e-8, 1e-4)
    diff = np.abs(got["flagged"].cpu().numpy() - cnt)
    assert diff.sum() <= 0.01 * cnt.sum() + 2
    assert got["max_rel_error"] == pytest.approx(rel.max(), rel=1e-3)


def test_eval_batch_host_concurrent_threads():
    """The host entry from several host threads at once (one library-owned staging buffer and
    stream per device, serialised by a lock): every call returns its own inputs' results."""
    import threading

    prob, x, mass, tag = _inputs("ground4_1m", 64)
    want = [prob.eval_batch_host(x[i:i + 1], mass[i:i + 1], None, outputs=("g", "jac")) for i in range(8)]
    got, errors = {}, []

    def worker(t):
        try:
            for rep in range(25):
                i = (t + rep) % 8
                r = prob.eval_batch_host(x[i:i + 1], mass[i:i + 1], None, outputs=("g", "jac"))
                for k in ("g", "jac"):
                    if not np.array_equal(r[k], want[i][k], equal_nan=True):
                        errors.append((t, rep, k))
            got[t] = True
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    assert len(got) == 4
