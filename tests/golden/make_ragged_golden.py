#!/usr/bin/env python3
"""Generate the ragged-batch golden fixtures (tests/golden/ragged_*.npz):
polygon and line formations at N in {3, 6, 24} ("C4
polygon/line assignments").

Each fixture holds B padded env states and what an observe of them must
return: the per-step assignment sigma, the reward -C[i][sigma_i] (fp32), node
features and the CSR edges (oracle/ragged_ref.py, fp32 mode). The assignment
is pinned twice at generation: oracle/lsa_ref.py's restatement and
scipy.optimize.linear_sum_assignment itself (the reference's dependency,
requirements.txt:101) must agree on every matrix, ties included. States:

  random   Philox layouts of the scenario (episode 0..3)
  onslot   agents exactly on the slots, in a permuted order (C[i][pi_i] = 0)
  centre   every agent at the formation centre (polygon) / the line's
           midpoint: every row equal — scipy's tie rules decide sigma
  mirror   agents in pairs at (x, +h) and (x, -h) about a horizontal line
           formation (identical cost rows: exact float32 ties, the kind that
           force the kernel's cold solve); polygon: coincident
           pairs (identical rows as well)

plus a short fp32 step chain (s_{t+1} = fp32(step_fp64(s_t))) from the random
states for the physics bar. Usage: python tests/golden/make_ragged_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
from scipy.optimize import linear_sum_assignment as scipy_lsa

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from oracle import ragged_ref as rr      # noqa: E402

CASES = [("polygon", 3), ("polygon", 6), ("polygon", 24), ("line", 3), ("line", 6), ("line", 24)]
KINDS = ("random", "random", "random", "onslot", "centre", "mirror", "mirror", "random")


def name_of(scenario, n):
    return f"ragged_{scenario}{n}"


def states(cfg, scn, n, seed):
    """[B, E_max, 2] fp32 padded positions of the fixture's envs."""
    rs = rr.RSpec(cfg)
    rng = np.random.default_rng(1000 * scn + n)
    B = len(KINDS)
    pos = np.zeros((B, rs.Emax, 2), np.float32)
    idx = rr.store_index(rs, scn, n)
    for b, kind in enumerate(KINDS):
        pc = rr.layout_env(cfg, b, b % 4, n, scn, seed)           # compact: agents, targets
        T = rr.n_targets(scn, n)
        if kind == "onslot":
            s = rr.slots(cfg, scn, n, pc[n:n + T])
            pc[:n] = s[rng.permutation(n)]
        elif kind == "centre":
            c = pc[n] if scn == rr.SCN_POLYGON else (pc[n] + pc[n + 1]) * np.float32(0.5)
            pc[:n] = c
        elif kind == "mirror":
            if scn == rr.SCN_LINE:
                pc[n] = np.array([-1.0, 0.25], np.float32)               # horizontal line at y = 0.25
                pc[n + 1] = np.array([1.0, 0.25], np.float32)
                for i in range(0, n - 1, 2):
                    x = np.float32(rng.uniform(-1, 1))
                    h = np.float32(rng.integers(51, 600) / 1024.0)   # 0.25 +- h exact in fp32
                    pc[i] = (x, np.float32(0.25) + h)
                    pc[i + 1] = (x, np.float32(0.25) - h)
                if n % 2:
                    pc[n - 1] = (np.float32(rng.uniform(-1, 1)), np.float32(0.25))
            else:
                for i in range(0, n - 1, 2):
                    pc[i + 1] = pc[i]                                     # identical rows
        pos[b, idx] = pc
    return pos


def observe_fixture(cfg, pos, vel, scn, n):
    rs = rr.RSpec(cfg)
    B = pos.shape[0]
    st = dict(pos=pos, vel=vel, step=np.zeros(B, np.int32), episode=np.zeros(B, np.int32),
              ep_acc=np.zeros((B, 2)), ep_last=np.zeros((B, 2)), n=np.full(B, n, np.int32),
              scn=np.full(B, scn, np.int32), seed=int(cfg.seed))
    ob = rr.observe(cfg, st)
    reward = np.zeros((B, rs.Nmax), np.float32)
    for b in range(B):
        pc = pos[b, rr.store_index(rs, scn, n)]
        sigma, C = rr.assignment(cfg, scn, n, pc)
        sp_rows, sp_cols = scipy_lsa(C.astype(np.float64))
        assert np.array_equal(sp_rows, np.arange(n)) and np.array_equal(sp_cols, sigma), (scn, n, b)
        assert np.array_equal(ob["assign"][b, :n], sigma)
        reward[b, :n] = -C[np.arange(n), sigma]
    return dict(assign=ob["assign"], reward=reward, node_feat=ob["node_feat"], edge_ptr=ob["edge_ptr"],
                edge_index=ob["edge_index"], edge_attr=ob["edge_attr"])


def chain(cfg, pos, vel, actions):
    """fp32 chain of one-step fp64 expectations from the random states."""
    rs = rr.RSpec(cfg)
    B = pos.shape[0]
    st = dict(pos=pos, vel=vel, step=np.zeros(B, np.int32), episode=np.zeros(B, np.int32),
              ep_acc=np.zeros((B, 2)), ep_last=np.zeros((B, 2)), n=np.full(B, cfg.n_agents, np.int32),
              scn=np.full(B, cfg.scenario, np.int32), seed=int(cfg.seed))
    out = {k: [] for k in ("pos", "vel", "next_pos", "next_vel")}
    for t in range(actions.shape[0]):
        nst, _ = rr.step(cfg, st, actions[t], 1, np.float64)
        out["pos"].append(st["pos"].astype(np.float32))
        out["vel"].append(st["vel"].astype(np.float32))
        out["next_pos"].append(nst["pos"])
        out["next_vel"].append(nst["vel"])
        st = dict(nst, pos=nst["pos"].astype(np.float32), vel=nst["vel"].astype(np.float32))
    return {k: np.asarray(v) for k, v in out.items()}


def build(scenario, n):
    seed = 17
    cfg = rr.make_cfg(scenario=scenario, n_agents=n, n_envs=len(KINDS), seed=seed, episode_length=10**6)
    scn = int(cfg.scenario)
    pos = states(cfg, scn, n, seed)
    rng = np.random.default_rng(7 * n + scn)
    vel = rng.normal(scale=0.2, size=(len(KINDS), n, 2)).astype(np.float32)
    d = dict(pos=pos, vel=vel, kinds=np.array([KINDS.index(k) for k in KINDS], np.int32),
             cfg_scenario=np.int32(scn), cfg_n_agents=np.int32(n), cfg_n_envs=np.int32(len(KINDS)),
             cfg_seed=np.int64(seed))
    d.update(observe_fixture(cfg, pos, vel, scn, n))
    rand = np.array([k == "random" for k in KINDS])
    actions = rng.integers(0, 5, size=(4, len(KINDS), n)).astype(np.int32)
    ch = chain(cfg, pos, vel, actions)
    d.update({"chain_" + k: v for k, v in ch.items()})
    d["chain_actions"] = actions
    d["chain_envs"] = rand
    return d


def main():
    for scenario, n in CASES:
        d = build(scenario, n)
        np.savez_compressed(HERE / f"{name_of(scenario, n)}.npz", **d)
        print(name_of(scenario, n), {k: v.shape for k, v in d.items() if hasattr(v, "shape") and v.ndim})


if __name__ == "__main__":
    main()
