#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no fixtures or tests and its source is
absent, so these vectors come from this repo's oracle (oracle/batch_ref.py,
cross-checked against oracle/mpe_ref.py and pinned by the Philox KATs and the
analytic KATs). They freeze the oracle's behaviour (CPU test
test_golden.py::test_oracle_reproduces_fixtures) and travel to the GPU box,
where the HIP path is checked against them without importing anything that
needs /root/reference.

Every fixture is a chain of fp32 states: s_{t+1} = fp32(step_fp64(s_t)); the
expected values are the fp64 step from the fp32 state s_t. ``margin`` is the
smallest relative distance of any pair predicate (collision / radius) from
its threshold at the post-step state: integer outputs are compared exactly
when it exceeds the fp32 noise floor.

Usage: python tests/golden/make_golden.py   (writes *.npz next to this file)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from oracle import batch_ref as br           # noqa: E402
from oracle.philox import philox4x32_10      # noqa: E402


def margins(cfg, pos):
    """min over pairs of |d2 - thr| / thr for the collision and radius predicates."""
    sp = br.Spec(cfg, np.float64)
    pos = pos.astype(np.float64)
    d2 = ((pos[:, :, None, :] - pos[:, None, :, :]) ** 2).sum(-1)
    E = sp.E
    m = np.inf
    inAO = sp.etype != br.ENT_GOAL
    sizes = np.where(sp.etype == br.ENT_AGENT, cfg.agent_size,
                     np.where(sp.etype == br.ENT_GOAL, cfg.goal_size, cfg.obstacle_size))
    off = ~np.eye(E, dtype=bool)
    ao = (inAO[:, None] & inAO[None, :]) & off
    R2 = cfg.sense_radius ** 2
    m = min(m, float(np.min(np.abs(d2[:, ao] - R2) / R2)) if ao.any() else np.inf)
    ag = sp.etype == br.ENT_AGENT
    col = (ag[:, None] & inAO[None, :]) & off
    thr = (sizes[:, None] + sizes[None, :]) ** 2
    if col.any():
        m = min(m, float(np.min(np.abs(d2[:, col] - thr[col]) / thr[col])))
    return m


def chain(cfg, pos, vel, actions, fmt):
    """Roll a fixture chain; returns dict of stacked arrays."""
    T = actions.shape[0]
    out = {k: [] for k in ("pos", "vel", "next_pos", "next_vel", "reward", "cost", "margin",
                           "edge_count")}
    for t in range(T):
        p64, v64 = br.physics(cfg, pos.astype(np.float64), vel.astype(np.float64), actions[t], fmt)
        r, c = br.reward_cost(cfg, p64, np.float64)
        ptr, _, _ = br.edges(cfg, p64, np.float64)
        out["pos"].append(pos)
        out["vel"].append(vel)
        out["next_pos"].append(p64)
        out["next_vel"].append(v64)
        out["reward"].append(r)
        out["cost"].append(c)
        out["margin"].append(margins(cfg, p64))
        out["edge_count"].append(np.diff(ptr))
        pos, vel = p64.astype(np.float32), v64.astype(np.float32)
    return {k: np.asarray(v) for k, v in out.items()}


CASES = {}


def case(name):
    def deco(fn):
        CASES[name] = fn
        return fn
    return deco


@case("c1_nav3")
def _c1():
    """BASELINE configs[0]: 3 agents, 1 env, 100-step episodes, 4 seeds (stacked as B=4)."""
    cfg = br.make_cfg(n_agents=3, n_envs=4, seed=0)
    pos = np.concatenate([br.layout(cfg, [0], [0], seed) for seed in range(4)])
    vel = np.zeros((4, 3, 2), np.float32)
    x0, _, _, _ = philox4x32_10(np.arange(100 * 4 * 3), 0, 0, 1, 1234, 0)
    actions = (x0 % 5).astype(np.int32).reshape(100, 4, 3)
    return cfg, pos, vel, actions, 1


@case("contact_crowd")
def _crowd():
    """Contact-heavy: 6 agents + 4 obstacles packed in a 0.35 box, fast velocities."""
    cfg = br.make_cfg(n_agents=6, n_obstacles=4, n_envs=8, seed=0)
    rng = np.random.default_rng(42)
    pos = rng.uniform(-0.35, 0.35, size=(8, cfg.n_agents * 2 + 4, 2)).astype(np.float32)
    vel = rng.normal(scale=0.5, size=(8, 6, 2)).astype(np.float32)
    actions = rng.integers(0, 5, size=(10, 8, 6)).astype(np.int32)
    return cfg, pos, vel, actions, 1


@case("nav24_snapshot")
def _n24():
    cfg = br.make_cfg(n_agents=24, n_envs=2, seed=5)
    pos = br.layout(cfg, [0, 1], [3, 3], 5)
    vel = np.random.default_rng(2).normal(scale=0.3, size=(2, 24, 2)).astype(np.float32)
    oh = np.eye(5, dtype=np.float32)[np.random.default_rng(3).integers(0, 5, size=(3, 2, 24))]
    return cfg, pos, vel, oh, 0


@case("nav96_snapshot")
def _n96():
    cfg = br.make_cfg(n_agents=96, n_envs=1, seed=9)
    pos = br.layout(cfg, [0], [0], 9)
    vel = np.zeros((1, 96, 2), np.float32)
    a = np.random.default_rng(4).uniform(-1, 1, size=(2, 1, 96, 2)).astype(np.float32)
    return cfg, pos, vel, a, 2


@case("clamp_obstacle_free")
def _clamp():
    cfg = br.make_cfg(n_agents=5, n_obstacles=0, n_envs=3, max_speed=0.4, seed=0)
    rng = np.random.default_rng(7)
    pos = rng.uniform(-1, 1, size=(3, 10, 2)).astype(np.float32)
    vel = rng.normal(size=(3, 5, 2)).astype(np.float32)
    actions = rng.integers(0, 5, size=(6, 3, 5)).astype(np.int32)
    return cfg, pos, vel, actions, 1


CFG_KEYS = ("n_agents", "n_obstacles", "n_envs", "seed", "max_speed", "world_half")


def build(name):
    cfg, pos, vel, actions, fmt = CASES[name]()
    d = chain(cfg, pos, vel, actions, fmt)
    d["actions"] = actions
    d["fmt"] = np.int32(fmt)
    for k in CFG_KEYS:
        d["cfg_" + k] = np.asarray(getattr(cfg, k))
    return d


def layout_vectors():
    """Philox layouts (bit-exact) for a few (seed, env, episode) keys."""
    keys = [(0, 0, 0), (0, 7, 3), (1234, 8191, 0), (2**40 + 5, 3, 99)]
    cfg = br.make_cfg(n_agents=24)
    pos = np.stack([br.layout(cfg, [e], [ep], s)[0] for s, e, ep in keys])
    return dict(keys=np.array(keys, dtype=np.uint64), pos=pos)


def main():
    for name in CASES:
        d = build(name)
        np.savez_compressed(HERE / f"{name}.npz", **d)
        print(name, {k: v.shape for k, v in d.items() if hasattr(v, "shape") and v.ndim})
    np.savez_compressed(HERE / "layout_vectors.npz", **layout_vectors())


if __name__ == "__main__":
    main()
