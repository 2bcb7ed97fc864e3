"""On-device rollout buffer (gsmarl_amd.rollout):
redirected outputs (gsm_step_into / gsm_graph_capture_into) must equal what a
plain env produces with the same actions, bit for bit, for every slot; edge
overflow truncates without writing out of bounds; graph_batch slices match."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pair(**kw):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    return GpuBatchEnv(EnvConfig(**kw), DEV), GpuBatchEnv(EnvConfig(**kw), DEV)


def _check_slot(buf, t, out, B):
    n = int(out["edge_ptr"][B])
    assert n <= buf.cap
    for k in ("node_feat", "reward", "cost", "done", "edge_ptr"):
        assert torch.equal(getattr(buf, k)[t], out[k]), (t, k)
    assert torch.equal(buf.edge_index[t][:, :n], out["edge_index"][:, :n]), t
    assert torch.equal(buf.edge_attr[t][:n], out["edge_attr"][:n]), t


@pytest.mark.parametrize("kw", [dict(n_agents=24, n_envs=64), dict(n_agents=3, n_envs=100),
                                dict(n_agents=80, n_envs=6), dict(scenario="mixed", n_agents=12, n_envs=48)])
def test_eager_rollout_matches_plain_env(kw):
    from gsmarl_amd import GraphRolloutBuffer
    kw = dict(kw, seed=4, episode_length=7)
    env, ref = _pair(**kw)
    buf = GraphRolloutBuffer(env, episode_length=10)
    buf.reset(seed=4)
    out = ref.reset(seed=4)
    _check_slot(buf, 0, out, env.B)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    for t in range(10):
        a = torch.randint(0, 5, (env.B, env.N), dtype=torch.int32, device=DEV, generator=g)
        buf.insert(a)
        out = ref.step(a)
        torch.cuda.synchronize()
        _check_slot(buf, t + 1, out, env.B)
        if buf.ragged:
            assert torch.equal(buf.assign[t + 1], out["assign"])
    # the env state advanced exactly like the reference env's
    assert torch.equal(env.t["pos"], ref.t["pos"]) and torch.equal(env.t["vel"], ref.t["vel"])
    assert int(buf.done[1:].sum()) == env.B            # every env finished once (episode 7)
    assert not bool(buf.overflowed())
    buf.after_update()
    assert torch.equal(buf.node_feat[0], buf.node_feat[10])
    env.close()
    ref.close()


@pytest.mark.parametrize("N,B,T", [(24, 128, 9), (24, 130, 8), (3, 100, 1), (3, 100, 2), (5, 37, 7), (80, 6, 5)])
def test_graph_rollout_matches_eager(N, B, T):
    """The graph chain (segmented configs: lagged emission, slot j's edges
    written by step j+1's kernel) equals eager step_into slot by slot."""
    from gsmarl_amd import GraphRolloutBuffer
    env, ref = _pair(n_agents=N, n_envs=B, seed=2, episode_length=6)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    gb = GraphRolloutBuffer(env, episode_length=T)
    eb = GraphRolloutBuffer(ref, episode_length=T)
    gb.reset(seed=2)
    gb.capture(acts)
    # compiled segmented shapes and tile shapes run the episode as one fused
    # rollout launch writing slot j at base + j * stride
    assert env.graph_is_rollout(0) == (N in (3, 24, 80))
    gb.replay()
    assert not env.roll_gave_up()
    eb.reset(seed=2)
    for t in range(T):
        eb.insert(acts[t])
    torch.cuda.synchronize()
    for k in ("node_feat", "reward", "cost", "done", "edge_ptr", "edge_count", "actions"):
        assert torch.equal(getattr(gb, k), getattr(eb, k)), k
    for t in range(T + 1):
        n = int(gb.edge_ptr[t, B])
        assert torch.equal(gb.edge_index[t][:, :n], eb.edge_index[t][:, :n])
        assert torch.equal(gb.edge_attr[t][:n], eb.edge_attr[t][:n])
    env.close()
    ref.close()


def test_edge_overflow_is_truncated():
    from gsmarl_amd import GraphRolloutBuffer
    env, ref = _pair(n_agents=24, n_envs=32, seed=5)
    buf = GraphRolloutBuffer(env, episode_length=2, edges_per_env=8)    # far below the ~90 needed
    buf.reset(seed=5)
    out = ref.reset(seed=5)
    torch.cuda.synchronize()
    assert bool(buf.overflowed())
    assert torch.equal(buf.edge_ptr[0], out["edge_ptr"])                 # true offsets kept
    cap = buf.cap
    assert torch.equal(buf.edge_index[0], out["edge_index"][:, :cap])    # the prefix that fits
    # sampling a truncated env is a clear error, not a device-side index assert
    last = torch.tensor([31])
    with pytest.raises(ValueError, match="capacity"):
        buf.graph_batch(torch.tensor([0]), last)
    fits = int((buf.edge_ptr[0, 1:] <= cap).nonzero()[0].item()) if bool((buf.edge_ptr[0, 1:] <= cap).any()) else None
    if fits is not None:
        buf.graph_batch(torch.tensor([0]), torch.tensor([fits]))
    env.close()
    ref.close()


@pytest.mark.parametrize("N,B", [(24, 32), (3, 50)])
def test_graph_chain_overflow_is_truncated(N, B):
    """A rollout graph into slots far too small: every slot keeps its
    true CSR offsets and exactly the prefix of edges that fits; no slot's
    emission spills into another slot (each is checked against a plain env)."""
    from gsmarl_amd import GraphRolloutBuffer
    env, ref = _pair(n_agents=N, n_envs=B, seed=6, episode_length=3)
    T = 5
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    buf = GraphRolloutBuffer(env, episode_length=T, edges_per_env=2)
    buf.reset(seed=6)
    buf.capture(acts)
    assert env.graph_is_rollout(0)   # the rollout launch truncates exactly as the chain does
    buf.replay()
    assert not env.roll_gave_up()
    outs = [ref.reset(seed=6)]
    outs[0] = {k: v.clone() for k, v in outs[0].items()}
    for t in range(T):
        o = ref.step(acts[t])
        outs.append({k: v.clone() for k, v in o.items()})
    torch.cuda.synchronize()
    assert bool(buf.overflowed())
    cap = buf.cap
    for t in range(T + 1):
        assert torch.equal(buf.edge_ptr[t], outs[t]["edge_ptr"]), t
        assert torch.equal(buf.edge_index[t][0], outs[t]["edge_index"][0, :cap]), t
        assert torch.equal(buf.edge_index[t][1], outs[t]["edge_index"][1, :cap]), t
        assert torch.equal(buf.edge_attr[t], outs[t]["edge_attr"][:cap]), t
    env.close()
    ref.close()


def test_graph_batch_and_returns():
    from gsmarl_amd import GraphRolloutBuffer
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    env = GpuBatchEnv(EnvConfig(n_agents=6, n_envs=20, seed=8, episode_length=4), DEV)
    buf = GraphRolloutBuffer(env, episode_length=5)
    buf.reset(seed=8)
    for t in range(5):
        buf.insert(torch.randint(0, 5, (20, 6), dtype=torch.int32, device=DEV))
    t_idx = torch.tensor([0, 3, 5, 5, 1])
    b_idx = torch.tensor([7, 0, 19, 2, 7])
    g = buf.graph_batch(t_idx, b_idx)
    E = env.E
    for k, (t, b) in enumerate(zip(t_idx.tolist(), b_idx.tolist())):
        lo, hi = int(buf.edge_ptr[t, b]), int(buf.edge_ptr[t, b + 1])
        ref_src = buf.edge_index[t, 0, lo:hi].long() - b * E + k * E
        ref_dst = buf.edge_index[t, 1, lo:hi].long() - b * E + k * E
        s0, s1 = int(g["ptr"][k]), int(g["ptr"][k + 1])
        assert torch.equal(g["edge_index"][0, s0:s1], ref_src) and torch.equal(g["edge_index"][1, s0:s1], ref_dst)
        assert torch.equal(g["node_feat"][k * E:(k + 1) * E], buf.node_feat[t, b])
    assert int(g["edge_index"].min()) >= 0 and int(g["edge_index"].max()) < len(t_idx) * E
    v = torch.zeros(6, 20, 6, device=DEV)
    ret = buf.compute_returns(v, gamma=0.5, gae_lambda=1.0)
    # zero values, lambda 1: discounted reward-to-go cut at episode ends
    r, m = buf.rewards, buf.masks
    exp = torch.zeros_like(r)
    acc = torch.zeros_like(r[0])
    for t in reversed(range(5)):
        acc = r[t] + 0.5 * m[t + 1] * acc
        exp[t] = acc
    assert torch.allclose(ret, exp, atol=1e-5)
    env.close()
