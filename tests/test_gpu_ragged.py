"""Ragged HIP path (polygon / line / mixed, per-env N) vs oracle/ragged_ref.py,
through the C ABI.

Bars: reset layouts, env shapes, node features, LSA assignments, collision
costs, edge_ptr and edge_index bit-exact (the fp32-mode oracle evaluated on the
kernel's own fp32 positions; the assignment through oracle/lsa_ref.py, itself
pinned to scipy); positions/velocities within 1e-6 of the fp64 oracle stepped
from the identical state; rewards bit-exact for polygon/line (-C[i][sigma_i]
is the same fp32 value) and within 2 ulp for navigation and shared sums.
"""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

from oracle import ragged_ref as rr
from parity_tol import check_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _renv(**kw):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    cfg = EnvConfig(**kw)
    keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
    rcfg = rr.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in keys})
    return GpuBatchEnv(cfg, DEV), rcfg


def _np(t):
    return t.detach().cpu().numpy()


def _ostate(env, rcfg):
    sh = _np(env.t["env_shape"])
    return dict(pos=_np(env.t["pos"]), vel=_np(env.t["vel"]), step=_np(env.t["step_count"]).copy(),
                episode=_np(env.t["episode"]).copy(), ep_acc=_np(env.t["ep_acc"]).astype(np.float64),
                ep_last=_np(env.t["ep_last"]).astype(np.float64), n=sh & 0xFF, scn=sh >> 8,
                seed=int(rcfg.seed))




def check_observation(env, rcfg, out):
    st = _ostate(env, rcfg)
    ob = rr.observe(rcfg, st)
    assert np.array_equal(_np(out["edge_ptr"]), ob["edge_ptr"]), "edge_ptr"
    assert np.array_equal(_np(out["edge_index"]), ob["edge_index"]), "edge_index"
    assert np.allclose(_np(out["edge_attr"]), ob["edge_attr"], rtol=2.5e-7, atol=0), "edge_attr"
    assert np.array_equal(_np(out["assign"]), ob["assign"]), "assign"
    assert np.array_equal(_np(out["node_feat"]), ob["node_feat"]), "node_feat"
    return st


def check_reward_cost(env, rcfg, out, envs=None):
    st = _ostate(env, rcfg)
    rs = rr.RSpec(rcfg)
    reward, cost = _np(out["reward"]), _np(out["cost"])
    for b in (range(env.B) if envs is None else envs):
        n, scn, pc = rr._compact(rs, st, b)
        r, c, _ = rr.reward_cost_env(rcfg, scn, n, pc, np.float32)
        assert np.array_equal(cost[b, :n], c), ("cost", b)
        assert np.all(cost[b, n:] == 0) and np.all(reward[b, n:] == 0)
        if scn != rr.SCN_NAV and not rcfg.shared_reward:
            assert np.array_equal(reward[b, :n], r), ("reward", b)
        else:
            assert np.allclose(reward[b, :n], r, rtol=3e-7, atol=1e-6), ("reward", b)


CASES = [("polygon", 3, 3, 64), ("polygon", 24, 24, 256), ("line", 5, 5, 100), ("line", 1, 1, 8),
         ("polygon", 1, 1, 8), ("mixed", 24, 3, 512), ("mixed", 32, 1, 300)]


@pytest.mark.parametrize("scenario,N,nmin,B", CASES)
def test_reset_bit_exact(scenario, N, nmin, B):
    env, rcfg = _renv(scenario=scenario, n_agents=N, n_agents_min=nmin, n_envs=B, seed=21)
    out = env.reset(seed=21)
    torch.cuda.synchronize()
    ref = rr.new_state(rcfg, seed=21)
    n, scn = rr.env_shapes(rcfg, 21)
    assert np.array_equal(_np(out["n_agents_env"]), n) and np.array_equal(_np(out["scenario_env"]), scn)
    assert np.array_equal(_np(env.t["pos"]), ref["pos"]), "layout"
    assert np.all(_np(env.t["episode"]) == 0)
    check_observation(env, rcfg, out)
    check_reward_cost(env, rcfg, out)
    env.close()


@pytest.mark.parametrize("scenario,N,nmin,B", CASES)
@pytest.mark.parametrize("fmt", ["index", "onehot"])
def test_step_parity(scenario, N, nmin, B, fmt):
    env, rcfg = _renv(scenario=scenario, n_agents=N, n_agents_min=nmin, n_envs=B, seed=4)
    env.reset(seed=4)
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    for t in range(3):
        idx = torch.randint(0, 5, (B, N), device=DEV, generator=g, dtype=torch.int32)
        a = idx if fmt == "index" else torch.nn.functional.one_hot(idx.long(), 5).float()
        prev = _ostate(env, rcfg)
        out = env.step(a)
        torch.cuda.synchronize()
        st64, _ = rr.step(rcfg, prev, _np(a), 1 if fmt == "index" else 0, np.float64)
        got_p, got_v = _np(env.t["pos"]).astype(np.float64), _np(env.t["vel"]).astype(np.float64)
        check_state(got_p, st64["pos"], "pos")
        check_state(got_v, st64["vel"], "vel")
        check_observation(env, rcfg, out)
        check_reward_cost(env, rcfg, out)
    env.close()


@pytest.mark.parametrize("shared", [False, True])
def test_rollout_with_auto_reset(shared):
    B, N = 192, 24
    env, rcfg = _renv(scenario="mixed", n_agents=N, n_envs=B, seed=8, episode_length=6, shared_reward=shared)
    env.reset(seed=8)
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    for t in range(14):
        a = torch.randint(0, 5, (B, N), device=DEV, generator=g, dtype=torch.int32)
        prev = _ostate(env, rcfg)
        out = env.step(a)
        torch.cuda.synchronize()
        st64, ob64 = rr.step(rcfg, prev, _np(a), 1, np.float64)
        done = _np(out["done"])
        assert np.array_equal(done, ob64["done"])
        assert np.array_equal(_np(env.t["episode"]), st64["episode"])
        assert np.array_equal(_np(env.t["step_count"]), st64["step"])
        got_p = _np(env.t["pos"]).astype(np.float64)
        check_state(got_p, st64["pos"], f"pos t={t}")
        check_observation(env, rcfg, out)
        live = np.nonzero(done == 0)[0]
        check_reward_cost(env, rcfg, out, envs=live)
        if done.any():
            assert np.allclose(_np(env.t["ep_last"])[done == 1], st64["ep_last"][done == 1], rtol=1e-5, atol=1e-3)
    env.close()


@pytest.mark.parametrize("N", [4, 8, 17, 32])
def test_assignment_ties(N):
    """Tie-heavy states set by hand: stacked agents (identical rows), agents on
    the centre (all costs = r up to rounding), agents exactly on slots."""
    B = 6
    env, rcfg = _renv(scenario="polygon", n_agents=N, n_envs=B, seed=1)
    env.reset(seed=1)
    st = env.get_state()
    pos = st["pos"].clone()
    c = pos[:, N].clone()                      # polygon centres
    rng = np.random.default_rng(N)
    pos[0, :N] = pos[0, 0]                     # all stacked
    pos[1, :N] = c[1]                          # all on the centre
    pos[2, : N // 2] = pos[2, 0]               # half stacked
    sl = torch.from_numpy(rr.slots(rcfg, rr.SCN_POLYGON, N, _np(c[3:4]))).to(DEV)
    pos[3, :N] = sl[torch.from_numpy(rng.permutation(N)).to(DEV)]   # exactly on the slots
    pos[4, :N] = torch.round(pos[4, :N] * 4) / 4                      # coarse grid -> equal costs
    out = env.set_state(dict(pos=pos))
    torch.cuda.synchronize()
    stn = check_observation(env, rcfg, out)
    rs = rr.RSpec(rcfg)
    for b in range(B):
        n, scn, pc = rr._compact(rs, stn, b)
        _, C = rr.assignment(rcfg, scn, n, pc)
        _, col = scipy_lsa(C.astype(np.float64))
        assert np.array_equal(_np(out["assign"])[b, :n], col), b
    env.close()


def test_graph_replay_equals_eager():
    B, N, T = 256, 24, 25
    env, rcfg = _renv(scenario="mixed", n_agents=N, n_envs=B, seed=5, episode_length=10)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=5)
    for t in range(T):
        env.step(acts[t], sync_edges=False)
    eager = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=5)
    env.capture(acts, T)
    env.replay()
    torch.cuda.synchronize()
    n = int(eager["edge_ptr"][-1])
    for k in ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "assign", "env_shape",
              "edge_ptr", "ep_acc", "ep_last"):
        assert torch.equal(eager[k], env.t[k]), k
    assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n])
    env.close()


@pytest.mark.parametrize("scenario,N,B,T", [("mixed", 24, 8192, 7), ("mixed", 24, 257, 6), ("polygon", 12, 130, 5),
                                             ("line", 9, 64, 4)])
def test_lagged_chain_equals_eager(scenario, N, B, T):
    """Ragged graph chains emit step j's edges from step j+1's kernel (lagged
    emission, heaviest-first workgroup order for mixed): every state and output
    buffer as after eager steps and the two-kernel chain, odd and even chain
    lengths, partial workgroups, auto-resets (episode length 3); the bound
    edge-sum buffer then re-emits the same edges."""
    env, rcfg = _renv(scenario=scenario, n_agents=N, n_envs=B, seed=8, episode_length=3)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    keys = ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "done", "edge_count",
            "edge_ptr", "ep_acc", "ep_last", "row_mask", "assign", "env_shape")
    env.reset(seed=8)
    for t in range(T):
        env.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    eager = {k: v.clone() for k, v in env.t.items()}
    n = int(eager["edge_ptr"][-1])
    for kernels, slot in (("both", 0), ("unfused", 1)):
        env.reset(seed=8)
        env.capture(acts, T, slot=slot, kernels=kernels)
        env.t["edge_index"].fill_(-7)
        env.replay(slot)
        torch.cuda.synchronize()
        for k in keys:
            assert torch.equal(eager[k], env.t[k]), (kernels, k)
        assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n]), kernels
        assert torch.equal(eager["edge_attr"][:n], env.t["edge_attr"][:n]), kernels
        env.t["edge_index"].zero_()
        env.capture(None, 1, slot=3, kernels="emit")
        env.replay(3)
        torch.cuda.synchronize()
        assert torch.equal(eager["edge_ptr"], env.t["edge_ptr"]), kernels
        assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n]), kernels
    env.close()


def test_lagged_chain_every_step_into_rollout_slots():
    """capture_into on a mixed config (one ragged rollout launch, slot j's
    edges packed `depth` steps later): every slot equals eager step_into's."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
    B, N, T = 300, 24, 7
    kw = dict(scenario="mixed", n_agents=N, n_envs=B, seed=4, episode_length=4)
    env, ref = GpuBatchEnv(EnvConfig(**kw), DEV), GpuBatchEnv(EnvConfig(**kw), DEV)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    gb = GraphRolloutBuffer(env, episode_length=T)
    eb = GraphRolloutBuffer(ref, episode_length=T)
    gb.reset(seed=4)
    gb.capture(acts)
    assert env.graph_is_rollout(0)
    gb.replay()
    eb.reset(seed=4)
    for t in range(T):
        eb.insert(acts[t])
    torch.cuda.synchronize()
    for k in ("node_feat", "reward", "cost", "done", "edge_ptr", "edge_count", "assign"):
        assert torch.equal(getattr(gb, k), getattr(eb, k)), k
    for t in range(T + 1):
        n = int(gb.edge_ptr[t, B])
        assert torch.equal(gb.edge_index[t][:, :n], eb.edge_index[t][:, :n]), t
        assert torch.equal(gb.edge_attr[t][:n], eb.edge_attr[t][:n]), t
    assert not bool(gb.overflowed())
    env.close()
    ref.close()


def test_navigation_env_matches_navigation_batch():
    """A navigation env inside a mixed batch lays out exactly like the same
    env id of a plain navigation batch (different kernels, same contract)."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    env, rcfg = _renv(scenario="mixed", n_agents=24, n_envs=60, seed=2)
    env.reset(seed=2)
    n, scn = rr.env_shapes(rcfg, 2)
    pos = _np(env.t["pos"])
    rs = rr.RSpec(rcfg)
    for b in np.nonzero(scn == rr.SCN_NAV)[0][:4]:
        nav = GpuBatchEnv(EnvConfig(n_agents=int(n[b]), n_envs=1, env_base=int(b), seed=2), DEV)
        nav.reset(seed=2)
        assert np.array_equal(_np(nav.t["pos"])[0], pos[b, rr.store_index(rs, 0, int(n[b]))])
        nav.close()
    env.close()


def test_config_validation():
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    from gsmarl_amd._lib import GsmError
    with pytest.raises(GsmError):
        GpuBatchEnv(EnvConfig(scenario="polygon", n_agents=33, n_envs=2), DEV)
    with pytest.raises(GsmError):
        GpuBatchEnv(EnvConfig(scenario="mixed", n_agents=8, n_obstacles=3, n_envs=2), DEV)


def test_dropin_ragged_single_env():
    """Drop-in classes on ragged scenarios: per-agent lists of the env's own
    N_env agents; actions for N_env agents are padded with no-ops."""
    from gsmarl_amd import make_env
    env = make_env("simple_formation", "MultiAgentGraphConstrainEnv", device=DEV, n_agents=5, n_envs=1)
    obs, aid, node, adj = env.reset(seed=3)
    assert len(obs) == 5 and node[0].shape == (6, 7) and adj[0].shape == (6, 6)
    obs, aid, node, adj, rew, cost, done, info = env.step([np.eye(5)[1]] * 5)
    assert len(rew) == 5 and len(cost) == 5 and all(r <= 0 for r in rew)
    mixed = make_env("mixed", "MultiAgentConstrainEnv", device=DEV, n_agents=24, n_envs=1, env_base=4, seed=9)
    o = mixed.reset(seed=9)
    n, scn = rr.env_shapes(rr.make_cfg(scenario="mixed", n_agents=24, n_envs=1, env_base=4, seed=9), 9)
    assert len(o) == int(n[0]) == mixed.n_active
    o, r, c, d, inf = mixed.step(list(range(5)) * (int(n[0]) // 5) + [0] * (int(n[0]) % 5))
    assert len(r) == int(n[0]) and len(inf) == int(n[0])
    line = make_env("simple_line", "MultiAgentEnv", device=DEV, n_agents=4, n_envs=3)
    o = line.reset(seed=1)
    assert o.shape == (3, 4, 6)


@pytest.mark.parametrize("scenario,N,B", [("mixed", 24, 384), ("polygon", 12, 128), ("line", 9, 128)])
def test_warm_start_equals_cold(scenario, N, B):
    """The certified warm-started assignment (gsm.h lsa_v / lsa_col) gives
    exactly what the from-scratch scipy recurrence gives, step after step
    across auto-resets; the share of certified warm starts is reported."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    kw = dict(scenario=scenario, n_agents=N, n_envs=B, seed=12, episode_length=40)
    warm = GpuBatchEnv(EnvConfig(**kw), DEV)
    cold = GpuBatchEnv(EnvConfig(lsa_warm_start=False, **kw), DEV)
    warm.reset(seed=12)
    cold.reset(seed=12)
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    for t in range(90):
        a = torch.randint(0, 5, (B, N), dtype=torch.int32, device=DEV, generator=g)
        ow = warm.step(a)
        oc = cold.step(a)
        for k in ("assign", "reward", "cost", "node_feat", "edge_ptr"):
            assert torch.equal(ow[k], oc[k]), (t, k)
        assert torch.equal(warm.t["pos"], cold.t["pos"]) and torch.equal(warm.t["vel"], cold.t["vel"]), t
    hits, solves = warm.lsa_warm_stats()
    assert cold.lsa_warm_stats() == (0, 0)
    print(f"warm-start certified: {hits}/{solves} = {hits / max(solves, 1):.4f} ({scenario} N={N})")
    assert solves > 0 and hits / solves > 0.9
    # and the warm env still matches the oracle from its current state
    keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
    rcfg = rr.make_cfg(**{k: v for k, v in warm.cfg.to_dict().items() if k in keys})
    out = warm.observe()
    check_observation(warm, rcfg, out)
    warm.close()
    cold.close()
