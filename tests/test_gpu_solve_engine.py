"""The native solve engine (csrc/cpl_solver.hip) against itself and against the host restatement
(batch_ipm.py over the oracle's callbacks) on the paths the round-3 iteration added: IPOPT's
restoration phase, soft restoration and tiny steps.

* batch independence: every kernel of the iteration works on one instance per wave / workgroup and
  the KKT kernel is chosen by the system size alone (cpl_kkt.hip kkt_wave_kernel_for), so an
  instance solved alone and the same instance inside a batch of 64 take bitwise the same iterates;
* the restoration phase on the device: TestBasic's superquadric scenario from x = 0 enters it on its
  first iteration (the 0/0 cone Jacobian makes the first Newton step useless); the device solve
  ends like the host restatement (same status; the eval kernel and the oracle differ in the last
  bits of pow, so the trajectories are not bitwise the same and may settle in neighbouring local
  optima of this nonconvex problem).
"""
import numpy as np
import pytest
import torch

from centroidalplanner_amd.batch_ipm import STATUS_ACCEPTABLE, batch_ipm_solve
from centroidalplanner_amd.workload import solve_inputs, solve_problem

from test_batch_solve import OracleBatchEvaluator, _HESSIAN, _scenario


@pytest.mark.gpu
@pytest.mark.parametrize("hessian", ["exact", "limited-memory"])
def test_instance_alone_is_bitwise_the_instance_in_a_batch(hessian):
    prob = solve_problem().GetCplProblem()
    B = 64
    X0, mass = solve_inputs(prob, B, seed=31)
    dev = torch.device("cuda:0")
    full = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), max_iter=1000,
                           hessian=hessian)
    assert bool((full.status <= STATUS_ACCEPTABLE).all())
    for k in (0, 17, 63):
        one = batch_ipm_solve(prob, torch.as_tensor(X0[k:k + 1], device=dev), torch.as_tensor(mass[k:k + 1], device=dev),
                              max_iter=1000, hessian=hessian)
        assert int(one.status[0]) == int(full.status[k]) and int(one.iterations[0]) == int(full.iterations[k])
        assert torch.equal(one.x[0], full.x[k]) and torch.equal(one.y[0], full.y[k])


def _zero_start(prob):
    xl, xu, _, _ = prob.get_bounds_info()
    return np.clip(np.zeros(prob.n), xl, xu)


@pytest.mark.gpu
def test_small_batch_tail_launch_is_bitwise_the_large_batch_tail():
    """Above 256 rows the iteration's tail (the accept, the restoration entry with its least-squares
    multipliers, the counts) runs as three launches (k_resto_enter, cpl_kkt_qd_kernel, k_count1); at
    most 256 rows as one (k_tail_small).  An instance's iterates must not depend on which: TestBasic's
    superquadric scenario from x = 0 (the restoration phase from the first iteration) in a batch of
    300 — the three-launch tail until compaction — against the same instances solved alone."""
    prob, _, _ = _scenario("superquadric")
    x0 = _zero_start(prob)
    B = 300
    mass = np.linspace(80.0, 150.0, B)
    dev = torch.device("cuda:0")
    kw = dict(max_iter=600, hessian=_HESSIAN["superquadric"])
    full = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1)), device=dev), torch.as_tensor(mass, device=dev),
                           **kw)
    assert bool((full.restorations.cpu() > 0).all())  # every instance took the entry (on the 3-launch path)
    for k in (0, 151, 299):
        one = batch_ipm_solve(prob, torch.as_tensor(x0[None, :], device=dev), torch.as_tensor(mass[k:k + 1], device=dev),
                              **kw)
        assert int(one.status[0]) == int(full.status[k]) and int(one.iterations[0]) == int(full.iterations[k])
        assert int(one.restorations[0]) == int(full.restorations[k])
        assert torch.equal(one.x[0], full.x[k]) and torch.equal(one.y[0], full.y[k])


@pytest.mark.gpu
def test_restoration_phase_device_matches_host():
    prob, _, _ = _scenario("superquadric")
    x0 = _zero_start(prob)
    mass = np.array([100.0, 96.57673546])
    B = mass.size
    dev = torch.device("cuda:0")
    d = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1)), device=dev), torch.as_tensor(mass, device=dev),
                        max_iter=1000, hessian=_HESSIAN["superquadric"])
    h = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1))), torch.as_tensor(mass),
                        evaluator=OracleBatchEvaluator(prob), max_iter=1000, hessian=_HESSIAN["superquadric"])
    assert d.restorations is not None and d.restorations.dtype == torch.int64
    rd, rh = d.restorations.cpu().numpy(), h.restorations.numpy()
    # x = 0: the restoration phase from the first iteration on both paths (how many phases follow
    # depends on the trajectory, which the two evaluators' last-bit differences steer apart)
    assert (rh >= 1).all() and (rd >= 1).all()
    # both converge (optimal, or IPOPT's acceptable level: the trajectories are not bitwise the same)
    assert bool((h.status <= STATUS_ACCEPTABLE).all()) and bool((d.status.cpu() <= STATUS_ACCEPTABLE).all())
    # nonconvex (bilinear torque balance): trajectories that part in the restoration phase may end
    # in neighbouring local optima (0.6800 vs 0.6813 seen); both are certified optimal above
    np.testing.assert_allclose(d.objective.cpu().numpy(), h.objective.numpy(), rtol=1e-2)


@pytest.mark.gpu
def test_com_planner_from_zero_device_matches_host():
    """CoMPlanner from x = 0 (limited-memory): no restoration phase, converged on both paths."""
    prob, _, _ = _scenario("com")
    x0 = _zero_start(prob)
    mass = np.random.default_rng(3).uniform(80.0, 150.0, 8)
    B = mass.size
    dev = torch.device("cuda:0")
    d = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1)), device=dev), torch.as_tensor(mass, device=dev),
                        max_iter=1000, hessian="limited-memory")
    h = batch_ipm_solve(prob, torch.as_tensor(np.tile(x0, (B, 1))), torch.as_tensor(mass),
                        evaluator=OracleBatchEvaluator(prob), max_iter=1000, hessian="limited-memory")
    assert bool((d.status <= STATUS_ACCEPTABLE).all()) and bool((h.status <= STATUS_ACCEPTABLE).all())
    # converged to tol 1e-8 (scaled): objectives of ~3e-4 agree to the solver's tolerance
    np.testing.assert_allclose(d.objective.cpu().numpy(), h.objective.numpy(), rtol=1e-6, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("hessian,max_ls,max_soc,seed", [("limited-memory", 40, 4, 3), ("exact", 40, 4, 5),
                                                         ("limited-memory", 4, 1, 7), ("exact", 1, 2, 9)])
def test_fused_line_search_is_bitwise_the_stepwise_search(hessian, max_ls, max_soc, seed):
    """The whole line search in one launch (cpl_ls_backtrack_kernel FIRST: the first trial, its
    second-order corrections re-solved with the kept one-wave KKT factors, the backtracking) takes
    bitwise the iterates of the step-by-step search (trial point / eval / judge / SOC launches):
    every batch size then solves an instance the same way whichever path its size selects."""
    prob = solve_problem().GetCplProblem()
    B = 48
    X0, mass = solve_inputs(prob, B, seed=seed)
    dev = torch.device("cuda:0")
    X0t, mt = torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev)
    kw = dict(max_iter=1000, hessian=hessian, max_ls=max_ls, max_soc=max_soc)
    a = batch_ipm_solve(prob, X0t, mt, ls_kernel=2, **kw)
    b = batch_ipm_solve(prob, X0t, mt, ls_kernel=0, **kw)
    for k in ("x", "y", "status", "iterations", "objective", "restorations"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    if max_ls == 40:
        assert bool((a.status <= STATUS_ACCEPTABLE).all())


@pytest.mark.gpu
@pytest.mark.parametrize("B", [2047, 2048])
def test_fused_search_around_the_global_factor_threshold(B):
    """Batches on both sides of LS_GF_MIN (2 048): below it the fused search kernel runs the post-step
    prologue (the any-flags then cleared by the optimality kernel, several launches before the search
    sets them), from it on the second-order corrections re-solve from the KKT factors in global memory
    and the post-step kernel clears the flags.  Either way the iterates are bitwise the step-by-step
    search's (flag ownership: cpl_solver.hip, d_any)."""
    prob = solve_problem().GetCplProblem()
    X0, mass = solve_inputs(prob, B, seed=11)
    dev = torch.device("cuda:0")
    X0t, mt = torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev)
    kw = dict(max_iter=1000, hessian="limited-memory", max_ls=40, max_soc=4)
    a = batch_ipm_solve(prob, X0t, mt, ls_kernel=2, **kw)
    b = batch_ipm_solve(prob, X0t, mt, ls_kernel=0, **kw)
    for k in ("x", "y", "status", "iterations", "objective", "restorations"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert bool((a.status <= STATUS_ACCEPTABLE).all())


@pytest.mark.gpu
def test_ipopt_jacobian_regularisation_device_matches_host():
    """IPOPT's (2,2)-block regularisation of a rank-deficient Jacobian in the engine
    (cpl_solve_options.jacobian_regularization = 1: cpl_kkt_aug_kernel re-factorises the marked systems
    as the augmented system in (dw, s)) against the host restatement's opt-in form over the oracle
    (batch_ipm_solve(jacobian_regularization="ipopt")).  testSimpleProblem's Newton systems are rank
    deficient at every iteration (one contact); the R-pivot default crawls to "acceptable" in 388
    iterations on both, the regularised form converges (optimal in 12 on the host and the compiled
    restatement, test_oracle_solve.py).  The device's KKT kernels round differently from torch's
    factorisations, so the check is the outcome, the iteration count and the point, not the bits."""
    from test_oracle_solve import _testbasic

    prob, x0, mass = _testbasic("testSimpleProblem")
    dev = torch.device("cuda:0")
    kw = dict(max_iter=3000, hessian="limited-memory", jacobian_regularization="ipopt")
    g = batch_ipm_solve(prob, torch.as_tensor(x0[None], device=dev), torch.as_tensor(np.array([mass]), device=dev),
                        **kw)
    h = batch_ipm_solve(prob, torch.as_tensor(x0[None]), torch.as_tensor(np.array([mass])),
                        evaluator=OracleBatchEvaluator(prob, 1), **kw)
    print("device", int(g.status[0]), int(g.iterations[0]), float(g.objective[0]),
          "host", int(h.status[0]), int(h.iterations[0]), float(h.objective[0]))
    assert int(h.status[0]) == 0 and int(g.status[0]) == 0
    # measured: both optimal in 12 at objective 481 180.505 (profiles/r6/jacreg/)
    assert int(g.iterations[0]) <= 20 and int(g.iterations[0]) == int(h.iterations[0])
    assert float(g.objective[0]) == pytest.approx(float(h.objective[0]), rel=1e-9)
    np.testing.assert_allclose(g.x[0].cpu().numpy(), h.x[0].numpy(), rtol=0, atol=1e-6)
    # the default form on the device: the documented crawl
    p = batch_ipm_solve(prob, torch.as_tensor(x0[None], device=dev), torch.as_tensor(np.array([mass]), device=dev),
                        max_iter=3000, hessian="limited-memory")
    assert int(p.status[0]) == STATUS_ACCEPTABLE and int(p.iterations[0]) > 100


@pytest.mark.gpu
@pytest.mark.parametrize("hessian", ["exact", "limited-memory"])
def test_jacobian_regularisation_leaves_full_rank_solves_bitwise(hessian):
    """The solve workload's systems never lose rank, so with the regularisation switched on nothing is
    marked: the augmented kernel launches return at once and the iterates are bitwise the default's
    (the search then re-solves its second-order corrections stepwise — the same iterates bit for bit
    as the fused search, test_fused_line_search_is_bitwise_the_stepwise_search)."""
    prob = solve_problem().GetCplProblem()
    B = 64
    X0, mass = solve_inputs(prob, B, seed=31)
    dev = torch.device("cuda:0")
    args = (prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev))
    a = batch_ipm_solve(*args, max_iter=1000, hessian=hessian)
    b = batch_ipm_solve(*args, max_iter=1000, hessian=hessian, jacobian_regularization="ipopt")
    assert torch.equal(a.status, b.status) and torch.equal(a.iterations, b.iterations)
    assert torch.equal(a.x, b.x) and torch.equal(a.y, b.y)


@pytest.mark.gpu
@pytest.mark.parametrize("hessian", ["limited-memory", "exact"])
def test_ipopt_jacobian_regularisation_four_contacts_device_matches_host(hessian):
    """The regularised form on the one-wave KKT size (nw 47, m 30; the augmented system has 77 unknowns):
    TestBasic's ground scenario from x = 0, where A is rank deficient (every force 0) — the pivot form's
    first step is 1e9-sized along a direction set by rounding, so the two restatements part at once
    (test_oracle_solve.py); IPOPT's (2,2) block has no such ambiguity, and the device (the wave kernel
    marks, cpl_kkt_aug_kernel re-factorises, the second-order corrections re-solve through it) follows
    the host restatement's iterates, a batch of four masses at a time: the first iterate in both Hessian
    modes, the first three with the exact Hessian (measured: within 5e-13 of 307 at each).  With IPOPT's
    L-BFGS the iteration is chaotic here — on the host alone a 1e-13 relative change of the masses moves
    the second iterate by 1e-5 and the third by 15: the regularised step along the near-null direction
    scales as 1 / delta_c, the second-order corrections' too — so only its first iterate is compared
    (measured: 1e-13; the second 7e-4).  The corrections' re-solves refine once, as the restatements'
    do: without it the first iterate was 1.3e-7 off with the exact Hessian."""
    from test_oracle_solve import _testbasic

    prob, x0, _ = _testbasic("testGroundEnv")
    B = 4
    mass = np.array([100.0, 90.0, 110.0, 125.0])
    X0 = np.tile(x0, (B, 1))
    dev = torch.device("cuda:0")
    for k in ((1,) if hessian == "limited-memory" else (1, 2, 3)):
        kw = dict(max_iter=k, hessian=hessian, jacobian_regularization="ipopt")
        g = batch_ipm_solve(prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev), **kw)
        h = batch_ipm_solve(prob, torch.as_tensor(X0), torch.as_tensor(mass), evaluator=OracleBatchEvaluator(prob, B),
                            **kw)
        err = float((g.x.cpu() - h.x).abs().max())
        scale = float(h.x.abs().max())
        print(hessian, "iterate", k, "max |x_dev - x_host|", err, "scale", scale)
        assert err <= 1e-10 * max(1.0, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("hessian", ["limited-memory", "exact"])
def test_regularised_fused_search_is_bitwise_the_stepwise_search(hessian):
    """With the regularisation on, the fused search kernel re-solves a marked system's second-order
    corrections on one wave over the augmented factors (kkt_aug_resolve_wave, its own AUGR
    instantiation), the stepwise search through cpl_kkt_solve + cpl_kkt_aug_kernel on a workgroup: the
    same arithmetic, so the same iterates bit for bit — on TestBasic's ground scenario from x = 0, whose
    systems are rank deficient and whose first iteration takes a second-order correction."""
    from test_oracle_solve import _testbasic

    prob, x0, _ = _testbasic("testGroundEnv")
    B = 4
    mass = np.array([100.0, 90.0, 110.0, 125.0])
    dev = torch.device("cuda:0")
    args = (prob, torch.as_tensor(np.tile(x0, (B, 1)), device=dev), torch.as_tensor(mass, device=dev))
    kw = dict(max_iter=40, hessian=hessian, jacobian_regularization="ipopt")
    fused = batch_ipm_solve(*args, ls_kernel=2, **kw)
    step = batch_ipm_solve(*args, ls_kernel=0, **kw)
    assert torch.equal(fused.x, step.x) and torch.equal(fused.y, step.y)
    assert torch.equal(fused.iterations, step.iterations) and torch.equal(fused.status, step.status)


@pytest.mark.gpu
def test_regularised_search_split_by_marking_at_large_batches():
    """From LS_GF_MIN (2 048) on, with the regularisation on, the fused search runs as two launches: the
    default instantiation over the unmarked instances, the AUGR one over the marked (rank-deficient)
    ones.  A batch of 2 050 solve-workload instances, every 97th started from x = 0 (every force 0: A
    rank deficient) — the fused search bitwise the stepwise one over the whole batch; the instances from
    the workload's own starts (whose systems never lose rank) bitwise the pivot form's; the x = 0 ones
    not (the regularised step differs there)."""
    prob = solve_problem().GetCplProblem()
    B = 2050
    X0, mass = solve_inputs(prob, B, seed=23)
    xl, xu, _, _ = prob.get_bounds_info()
    zero = np.arange(0, B, 97)
    X0[zero] = np.clip(np.zeros(prob.n), xl, xu)
    dev = torch.device("cuda:0")
    args = (prob, torch.as_tensor(X0, device=dev), torch.as_tensor(mass, device=dev))
    kw = dict(max_iter=200, hessian="limited-memory")
    fused = batch_ipm_solve(*args, ls_kernel=2, jacobian_regularization="ipopt", **kw)
    step = batch_ipm_solve(*args, ls_kernel=0, jacobian_regularization="ipopt", **kw)
    for k in ("x", "y", "status", "iterations"):
        assert torch.equal(getattr(fused, k), getattr(step, k)), k
    pivot = batch_ipm_solve(*args, ls_kernel=2, **kw)
    rest = torch.as_tensor(np.setdiff1d(np.arange(B), zero), device=dev)
    assert torch.equal(fused.x[rest], pivot.x[rest]) and torch.equal(fused.iterations[rest], pivot.iterations[rest])
    zi = torch.as_tensor(zero, device=dev)
    assert not torch.equal(fused.x[zi], pivot.x[zi])


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_restoration_called_at_an_almost_feasible_point_device(k):
    """The engine's end of a failed line search (cpl_solver.hip fail_book): at an almost feasible point
    (theta <= 1e-2 tol) no restoration phase — the backup acceptable point restored and the solve
    stopped as acceptable there (RestoreAcceptablePoint), or without one a restoration failure.  The
    cases of test_oracle_solve.py (tests/golden/resto_acc_cases.json), where both CPU restatements reach
    the branch: without a backup point the device solve ends as a restoration failure; with one (case 1:
    IPOPT's default acceptable_tol) the same iteration restores an earlier iterate and ends as acceptable
    (measured: iteration 183 / 680 on the device, 129 / 1 414 and 176 / 903 in the compiled / host
    restatements — the degenerate trajectories part them by rounding; scripts/resto_acc_gpu_probe.py)."""
    from test_oracle_solve import _resto_case

    prob, x0, c = _resto_case(k)
    dev = torch.device("cuda:0")
    kw = dict(tol=c["tol"], max_iter=3000, hessian=c["hessian"])
    X0 = torch.as_tensor(x0[None], device=dev)
    mass = torch.as_tensor(np.array([prob.desc().mass]), device=dev)
    fail = batch_ipm_solve(prob, X0, mass, acceptable_tol=c["no_backup_tol"], **kw)
    back = batch_ipm_solve(prob, X0, mass, acceptable_tol=c["acceptable_tol"], **kw)
    assert int(fail.status[0]) == 4 and int(back.status[0]) == STATUS_ACCEPTABLE
    assert int(back.iterations[0]) == int(fail.iterations[0])
    assert not torch.equal(back.x, fail.x) and float(back.objective[0]) != float(fail.objective[0])
    # the same instance in a batch of 64 (perturbed starts around it) takes the branch at the same
    # iteration to the same point: the restore is per instance
    Xb = X0.repeat(64, 1)
    Xb[1:] += torch.as_tensor(np.random.default_rng(5).normal(0.0, 1e-3, (63, x0.size)), device=dev)
    batch = batch_ipm_solve(prob, Xb, mass.repeat(64), acceptable_tol=c["acceptable_tol"], **kw)
    assert int(batch.status[0]) == STATUS_ACCEPTABLE and int(batch.iterations[0]) == int(back.iterations[0])
    assert torch.equal(batch.x[0], back.x[0])
