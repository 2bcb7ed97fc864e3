"""Degenerate states on every kernel family,
through the C ABI: coincident collider pairs injected with set_state.

* the per-env flags (gsm_buffers.degenerate: 1 coincident pair with an agent,
  2 non-finite agent) equal the oracle's (batch_ref.degenerate /
  ragged_ref.degenerate_env) after observe and after each step;
* default mode: the coincident pair's force is guarded to zero — physics
  within 1e-6 of the fp64 oracle, everything finite;
* strict mode (EnvConfig.strict_degenerate): MPE's 0/0 force — NaN exactly
  where the oracle has NaN (both agents of the pair), spreading to every agent
  of the env on the next step; other envs unaffected; the ragged assignment
  of a NaN env is -1 and the launch terminates.
"""
import numpy as np
import pytest
import torch

from oracle import batch_ref as br
from oracle import ragged_ref as rr
from parity_tol import check_state

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

NAV_CASES = [  # (id, kwargs): seg G=1 (compile-time 24/24), seg G=4 (compile-time 3/3), runtime seg G=1
    # and G=4, tile with the symmetric sweep, tile with the row sweep
    ("seg_g1", dict(n_agents=24, n_envs=8)),
    ("seg_g4", dict(n_agents=3, n_envs=4096)),
    ("seg_rt_g1", dict(n_agents=5, n_envs=64)),
    ("seg_rt_g4", dict(n_agents=5, n_envs=4096)),
    ("tile_sym", dict(n_agents=40, n_envs=4)),
    ("tile_rows", dict(n_agents=200, n_envs=4)),   # symmetric-sweep LDS > 32 KB: the row sweep
]


def _np(t):
    return t.detach().cpu().numpy()


def _inject_nav(pos, N, E):
    """env 0: agent 1 on agent 0; env 1: agent 2 on obstacle 0; env 2 (if
    any): obstacle 1 on obstacle 0 only (not degenerate)."""
    pos = pos.copy()
    pos[0, 1] = pos[0, 0]
    pos[1, 2] = pos[1, 2 * N]
    if pos.shape[0] > 2:
        pos[2, 2 * N + 1] = pos[2, 2 * N]
    return pos


@pytest.mark.parametrize("strict", [False, True])
@pytest.mark.parametrize("case,kw", NAV_CASES, ids=[c[0] for c in NAV_CASES])
def test_navigation_degenerate(case, kw, strict):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    cfg = EnvConfig(seed=5, strict_degenerate=strict, **kw)
    ocfg = br.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in br.DEFAULTS})
    env = GpuBatchEnv(cfg, DEV)
    env.reset(seed=5)
    B, N, E = env.B, env.N, env.E
    st = {k: _np(v) for k, v in env.get_state().items()}
    st["pos"] = _inject_nav(st["pos"], N, E)
    out = env.set_state({"pos": torch.from_numpy(st["pos"])})
    torch.cuda.synchronize()
    want = br.degenerate(ocfg, st["pos"])
    assert want[:2].tolist() == [1, 1] and (B < 3 or want[2] == 0)
    assert np.array_equal(_np(out["degenerate"]), want)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    for t in range(2):
        pos0, vel0 = _np(env.t["pos"]), _np(env.t["vel"])
        a = torch.randint(0, 5, (B, N), dtype=torch.int32, device=DEV, generator=g)
        out = env.step(a)
        torch.cuda.synchronize()
        with np.errstate(invalid="ignore"):
            p64, v64 = br.physics(ocfg, pos0.astype(np.float64), vel0.astype(np.float64), _np(a), 1)
        pos1, vel1 = _np(env.t["pos"]), _np(env.t["vel"])
        check_state(pos1, p64, f"{case} pos t={t}")
        check_state(vel1, v64, f"{case} vel t={t}")
        assert np.array_equal(_np(out["degenerate"]), br.degenerate(ocfg, pos1)), t
        if strict:
            nan_agents = np.isnan(pos1[:, :N]).any(-1)
            if t == 0:   # the coincident pair's agents only
                assert nan_agents[0, :2].all() and not nan_agents[0, 2:].any()
                assert nan_agents[1, 2] and nan_agents[1].sum() == 1
            else:        # MPE evaluates every pair: the whole env
                assert nan_agents[:2].all()
            assert not nan_agents[2:].any()
            assert (_np(out["degenerate"])[:2] & 2).all()
        else:
            assert np.isfinite(pos1).all() and np.isfinite(vel1).all()
        # costs of the NaN agents are 0 (every comparison with NaN is false);
        # the fp32 oracle on the kernel's positions gives the same counts
        _, c32 = br.reward_cost(ocfg, pos1, np.float32)
        assert np.array_equal(_np(out["cost"]), c32)
    env.close()


@pytest.mark.parametrize("strict", [False, True])
@pytest.mark.parametrize("scenario,N,B", [("polygon", 6, 8), ("mixed", 12, 48)])
def test_ragged_degenerate(scenario, N, B, strict):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    cfg = EnvConfig(scenario=scenario, n_agents=N, n_envs=B, seed=6, strict_degenerate=strict)
    keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
    rcfg = rr.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in keys})
    env = GpuBatchEnv(cfg, DEV)
    env.reset(seed=6)
    rs = rr.RSpec(rcfg)
    sh = _np(env.t["env_shape"])
    pos = _np(env.t["pos"]).copy()
    pos[0, 1] = pos[0, 0]                                   # agents 0 and 1 coincide
    if scenario == "mixed":                                 # env 0 is a navigation env: agent 2 on obstacle 0
        assert sh[0] >> 8 == 0
        pos[0, 2] = pos[0, rs.Nmax + rs.Tmax]
    env.set_state({"pos": torch.from_numpy(pos)})
    torch.cuda.synchronize()

    def ostate():
        s = _np(env.t["env_shape"])
        return dict(pos=_np(env.t["pos"]), vel=_np(env.t["vel"]), step=_np(env.t["step_count"]).copy(),
                    episode=_np(env.t["episode"]).copy(), ep_acc=_np(env.t["ep_acc"]).astype(np.float64),
                    ep_last=_np(env.t["ep_last"]).astype(np.float64), n=s & 0xFF, scn=s >> 8, seed=6)

    ob = rr.observe(rcfg, ostate())
    assert ob["degenerate"][0] == 1 and not ob["degenerate"][1:].any()
    assert np.array_equal(_np(env.t["degenerate"]), ob["degenerate"])
    g = torch.Generator(device=DEV)
    g.manual_seed(2)
    for t in range(2):
        prev = ostate()
        a = torch.randint(0, 5, (B, N), dtype=torch.int32, device=DEV, generator=g)
        out = env.step(a)
        torch.cuda.synchronize()
        with np.errstate(invalid="ignore"):
            st64, _ = rr.step(rcfg, prev, _np(a), 1, np.float64)
        check_state(_np(env.t["pos"]), st64["pos"], f"{scenario} pos t={t}")
        check_state(_np(env.t["vel"]), st64["vel"], f"{scenario} vel t={t}")
        ob = rr.observe(rcfg, ostate())
        assert np.array_equal(_np(out["degenerate"]), ob["degenerate"]), t
        assert np.array_equal(_np(out["assign"]), ob["assign"]), t
        n0 = int(sh[0] & 0xFF)
        if strict:
            assert np.isnan(_np(env.t["pos"])[0, :2]).all()
            if sh[0] >> 8 != 0:                             # polygon/line env with NaN: no assignment
                assert (_np(out["assign"])[0, :n0] == -1).all()
                assert np.isnan(_np(out["reward"])[0, :n0]).all()
        else:
            assert np.isfinite(_np(env.t["pos"])).all()
        assert np.isfinite(_np(env.t["pos"])[1:]).all()
    env.close()
