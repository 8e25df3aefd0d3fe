"""Seeded synthetic instances of the BASELINE.json configurations.

Each instance is a random (CoM, mass, contact-set) point of one problem template:
  c ~ U([-0.2,0.2]^2 x [0.8,1.2]);  mass ~ U[20,150];
  F_i = f_n n_i + tangential, f_n ~ U[0.2,2]*m*9.81/N, |tangential| <= 0.8*mu*f_n
        (inside the friction cone: FrictionCone stays away from its 0/0 point);
  n_i = environment normal at p_i + N(0,1e-3), normalised;
  Ground: z_g=0.1, mu=0.5, p ~ U([-0.3,0.3]^2) x {z_g + U(-1e-3,1e-3)};
  Superquadric: C=(0,0,1), R=(0.3,0.3,10), P=(10,10,10), mu=0.5 (tests/TestBasic.cpp:150-157),
        p ~ U([-0.5,0.5]^2 x [0.5,1.5]) (:163-164), |p_k - C_k| >= 1e-3 unless stress=True;
  wrench = (100,0,0,0,0,100) (:95-99); F_thr = 0; mixed: even instances Ground, odd Superquadric.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._abi import ENV_GROUND, ENV_MIXED, ENV_NONE, ENV_SUPERQUADRIC
from .problem import CplProblem, Ground, MixedEnvironment, Superquadric

SQ_C = np.array([0.0, 0.0, 1.0])
SQ_R = np.array([0.3, 0.3, 10.0])
SQ_P = np.array([10.0, 10.0, 10.0])
GROUND_Z = 0.1
MU = 0.5
WRENCH = np.array([100.0, 0.0, 0.0, 0.0, 0.0, 100.0])


@dataclass(frozen=True)
class Config:
    name: str
    n_contacts: int
    env: str  # "ground" | "superquadric" | "mixed" | "none"
    batch: int
    config_id: int


# BASELINE.json "configs" (index = config_id - 1); configs[0] is the single-instance plumbing case
CONFIGS = {
    "ground4": Config("4-contact Ground env, batch=65,536", 4, "ground", 65536, 2),
    "sq8": Config("8-contact Superquadric env, batch=262,144", 8, "superquadric", 262144, 3),
    "mixed16": Config("16-contact mixed Ground+Superquadric, batch=1,048,576", 16, "mixed", 1048576, 4),
    "ground4_1m": Config("4-contact Ground env, batch=1,048,576 (north-star target)", 4, "ground", 1048576, 6),
    "none4": Config("4-contact no-environment (CoMPlanner) statics, batch=65,536", 4, "none", 65536, 7),
    # measurement aid: the Ground half of configs[3] on its own
    "ground16": Config("16-contact Ground env, batch=524,288 (the Ground half of configs[3])", 16, "ground", 524288, 8),
    "sq16": Config("16-contact Superquadric env, batch=524,288 (the Superquadric half of configs[3])", 16,
                   "superquadric", 524288, 9),
}


def make_problem(n_contacts: int, env: str, mass: float = 100.0, names=None) -> CplProblem:
    names = names or [f"contact{i + 1}" for i in range(n_contacts)]
    if env == "ground":
        e = Ground()
        e.SetGroundZ(GROUND_Z)
        e.SetMu(MU)
    elif env == "superquadric":
        e = Superquadric()
        e.SetParameters(SQ_C, SQ_R, SQ_P)
        e.SetMu(MU)
    elif env == "mixed":
        g = Ground()
        g.SetGroundZ(GROUND_Z)
        s = Superquadric()
        s.SetParameters(SQ_C, SQ_R, SQ_P)
        e = MixedEnvironment(g, s)
        e.SetMu(MU)
    elif env == "none":
        e = None
    else:
        raise ValueError(env)
    prob = CplProblem(names, mass, e)
    if e is None:
        prob.SetMu(MU)
    prob.SetManipulationWrench(WRENCH)
    return prob


def _sq_normal(p: np.ndarray) -> np.ndarray:
    """Outward-facing -grad f/|grad f| of the superquadric, as Superquadric::GetNormalValue."""
    d = p - SQ_C
    j = SQ_P / SQ_R ** SQ_P * np.sign(d) * np.abs(d) ** (SQ_P - 1)
    nrm = np.linalg.norm(j, axis=-1, keepdims=True)
    nrm = np.where(nrm == 0, 1.0, nrm)
    return -j / nrm


def generate(n_contacts: int, env: str, batch: int, seed: int, stress: bool = False):
    """Returns (x [B, n], mass [B], env_tag [B] uint8 or None) as host arrays."""
    rng = np.random.default_rng(seed)
    N, B = n_contacts, batch
    n = 3 + 9 * N
    x = np.empty((B, n))
    x[:, 0] = rng.uniform(-0.2, 0.2, B)
    x[:, 1] = rng.uniform(-0.2, 0.2, B)
    x[:, 2] = rng.uniform(0.8, 1.2, B)
    mass = rng.uniform(20.0, 150.0, B)
    if env == "mixed":
        tag = np.where(np.arange(B) % 2 == 0, ENV_GROUND, ENV_SUPERQUADRIC).astype(np.uint8)
    else:
        tag = None
    is_sq = (tag == ENV_SUPERQUADRIC) if tag is not None else np.full(B, env == "superquadric")
    for i in range(N):
        # position
        pg = np.stack([rng.uniform(-0.3, 0.3, B), rng.uniform(-0.3, 0.3, B),
                       GROUND_Z + rng.uniform(-1e-3, 1e-3, B)], axis=1)
        ps = np.stack([rng.uniform(-0.5, 0.5, B), rng.uniform(-0.5, 0.5, B), rng.uniform(0.5, 1.5, B)], axis=1)
        if not stress:
            d = ps - SQ_C
            small = np.abs(d) < 1e-3
            ps = np.where(small, SQ_C + np.where(d >= 0, 1e-3, -1e-3) + d, ps)
        p = np.where(is_sq[:, None], ps, pg)
        if env == "none":
            p = pg
        # normal
        en = np.where(is_sq[:, None], _sq_normal(p), np.array([0.0, 0.0, 1.0]))
        if env == "none":
            en = np.tile(np.array([0.0, 0.0, 1.0]), (B, 1))
        nv = en + rng.normal(0.0, 1e-3, (B, 3))
        nv /= np.linalg.norm(nv, axis=1, keepdims=True)
        # force inside the cone
        fn = rng.uniform(0.2, 2.0, B) * mass * 9.81 / N
        a = rng.normal(size=(B, 3))
        a -= (a * nv).sum(1, keepdims=True) * nv
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        ft = rng.uniform(0.0, 0.8 * MU, B) * fn
        F = fn[:, None] * nv + ft[:, None] * a
        x[:, 3 + 9 * i: 6 + 9 * i] = F
        x[:, 6 + 9 * i: 9 + 9 * i] = p
        x[:, 9 + 9 * i: 12 + 9 * i] = nv
    return x, mass, tag


def config_inputs(cfg: Config, batch: Optional[int] = None, stress: bool = False):
    prob = make_problem(cfg.n_contacts, cfg.env)
    x, mass, tag = generate(cfg.n_contacts, cfg.env, batch or cfg.batch, 0xC910 + cfg.config_id, stress=stress)
    return prob, x, mass, tag


# BASELINE.json configs[4]: the full solve loop, 4 contacts, 8,192 concurrent instances on one GPU
SOLVE_CONFIG = Config("Full solve loop with GPU eval callbacks, 4-contact Ground, 8,192 concurrent instances",
                      4, "ground", 8192, 5)


def solve_problem(n_contacts: int = 4, force_weight: float = 1.0):
    """The TestBasic ground scenario (tests/TestBasic.cpp:64-100: Ground z=0.1, mu=0.5, CoM weight 2,
    contact positions boxed to [-0.3,0.3]^2 x [0,1], wrench (100,0,0,0,0,100)) as the shared
    template of a batched solve.  force_weight: TestBasic sets 0 (forces then only constrained:
    a degenerate problem); the batched workload keeps the reference default 1
    (src/MinimizeCentroidalVariables.cpp:11-25)."""
    from .planner import CentroidalPlanner

    names = [f"contact{i + 1}" for i in range(n_contacts)]
    env = Ground()
    env.SetGroundZ(GROUND_Z)
    env.SetMu(MU)
    cpl = CentroidalPlanner(names, 100.0, env)
    cpl.SetCoMWeight(2.0)
    cpl.SetForceWeight(force_weight)
    for c in names:
        cpl.SetPosBounds(c, np.array([-0.3, -0.3, 0.0]), np.array([0.3, 0.3, 1.0]))
    cpl.SetManipulationWrench(WRENCH)
    return cpl


def solve_inputs(prob, batch: int, seed: int = 0xC910 + 5):
    """Per-instance robot masses U[80, 150] kg (feasible under the wrench: the friction needed for
    the lateral force and the yaw torque stays inside mu * m g) and a non-degenerate start per
    instance: CoM at its reference, F_i = (1, 1, m g / N), p_i on a circle of radius 0.2 at
    z = 0.05, n_i = (0, 0, 1) — clipped into the variable bounds.  Host arrays (X0 [B, n], mass [B])."""
    rng = np.random.default_rng(seed)
    N = len(prob.contact_names)
    mass = rng.uniform(80.0, 150.0, batch)
    x0 = np.zeros(prob.n)
    x0[0:3] = prob.GetCoMRef()
    X0 = np.tile(x0, (batch, 1))
    for i in range(N):
        ang = 2.0 * np.pi * (i + 0.125) / N
        X0[:, 3 + 9 * i] = 1.0
        X0[:, 4 + 9 * i] = 1.0
        X0[:, 5 + 9 * i] = mass * 9.81 / N
        X0[:, 6 + 9 * i: 9 + 9 * i] = [0.2 * np.cos(ang), 0.2 * np.sin(ang), 0.05]
        X0[:, 9 + 9 * i: 12 + 9 * i] = [0.0, 0.0, 1.0]
    xl, xu, _, _ = prob.get_bounds_info()
    return np.clip(X0, xl, xu), mass


__all__ = ["Config", "CONFIGS", "SOLVE_CONFIG", "make_problem", "generate", "config_inputs", "solve_problem",
           "solve_inputs", "ENV_NONE", "ENV_MIXED"]
