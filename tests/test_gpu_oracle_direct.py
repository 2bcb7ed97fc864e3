"""The vec-env (reference env_wrappers.py, SOURCES.txt:11)
and the graph rollout buffer (§8(f) #2, reference graph_separated_buffer.py,
SOURCES.txt:33) checked against the CPU oracle directly, not against the
library's own eager path.

* GpuGraphVecEnv (MAPPO vec-env contract, one-hot actions, numpy outputs,
  dense adjacency) is stepped beside B object-per-entity oracle envs
  (oracle/mpe_ref.GraphConstrainEnv, one per env thread, as the reference's
  subprocess workers hold one env each) fed the same actions, across two
  auto-resets. Each step the oracle envs start from the kernel's pre-step
  fp32 state (fp32 rounding would otherwise accumulate), and the physics,
  rewards, costs, dones, observations, node tables, dense adjacency, infos
  and episode totals are compared.
* A captured GraphRolloutBuffer episode (one HIP graph, outputs redirected
  into the slots) is replayed; every slot t+1 is checked against
  oracle/batch_ref.step from the state held in slot t.

State tolerance: tests/parity_tol.py (north_star's 1e-6).
"""
import numpy as np
import pytest
import torch

from oracle import batch_ref as br
from oracle import mpe_ref
from parity_tol import check_state

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _np(t):
    return t.detach().cpu().numpy()


def check_cost_vs_fp64(got, ref, pos, N, what):
    """Collision counts against the fp64 oracle's. They may differ only where
    a pair sits on the contact boundary d = dmin to within fp32 rounding —
    which MPE's defaults make systematic, not rare: an agent overlapping an
    immovable obstacle is pushed by c * (dmin - d) in the linear regime of the
    softplus, so after one step (dv = F dt, dx = v dt with c dt^2 = 1) it lands
    on d = dmin. The kernel's count is the fp32 squared predicate on its own
    positions (checked bit-exact against the fp32 oracle elsewhere)."""
    got, ref = np.asarray(got), np.asarray(ref)
    if np.array_equal(got, ref):
        return
    pos = np.asarray(pos, np.float64)
    No = pos.shape[0] - 2 * N
    coll = np.concatenate([pos[:N], pos[2 * N:]])
    dmin = np.concatenate([np.full(N, 0.1), np.full(No, 0.13)])
    for i in np.nonzero(got != ref)[0]:
        d = np.sqrt(((coll - pos[i]) ** 2).sum(-1))
        near = np.abs(d - dmin) < 2e-6
        near[i] = False
        assert near.any() and abs(got[i] - ref[i]) <= near.sum(), (what, i, got[i], ref[i])


def test_vec_env_against_oracle_envs():
    from gsmarl_amd import EnvConfig, GpuGraphVecEnv
    B, N, EL, T, seed = 16, 4, 5, 12, 3
    cfg = EnvConfig(n_agents=N, n_envs=B, episode_length=EL, seed=seed)
    vec = GpuGraphVecEnv(cfg, DEV, output="numpy", graph="dense")
    E = vec.batch.E
    ocfg = br.make_cfg(n_agents=N, seed=seed, episode_length=EL)
    orc = [mpe_ref.GraphConstrainEnv(ocfg, env_gid=b) for b in range(B)]

    def check_reset_obs(got, obs_n, what):
        # reset layouts are bit-exact (Philox), velocities zero; the goal-relative
        # columns are one fp32 rounding of the fp64 difference
        want = np.array(obs_n)
        assert np.array_equal(got[:, :4].astype(np.float64), want[:, :4]), what
        assert np.allclose(got[:, 4:], want[:, 4:], rtol=0, atol=2.5e-7), what

    obs, aid, node, adj = vec.reset(seed=seed)
    for b, o in enumerate(orc):
        obs_n, _, _, _ = o.reset(seed=seed)
        check_reset_obs(obs[b], obs_n, b)
    rng = np.random.default_rng(11)
    eye = np.eye(5, dtype=np.float32)
    ep_r = np.zeros(B)
    ep_c = np.zeros(B)
    resets = 0
    for t in range(T):
        pos0, vel0 = _np(vec.batch.t["pos"]), _np(vec.batch.t["vel"])
        for b, o in enumerate(orc):                     # start from the kernel's fp32 state
            o.set_state(pos0[b].astype(np.float64), vel0[b].astype(np.float64))
        a = eye[rng.integers(0, 5, size=(B, N))]        # one-hot [B, N, 5]
        obs, aid, node, adj, rew, cost, done, infos = vec.step(a)
        assert obs.shape == (B, N, 6) and node.shape == (B, N, E, 7) and adj.shape == (B, N, E, E)
        assert np.array_equal(aid[:, :, 0], np.tile(np.arange(N), (B, 1)))
        pos1, vel1 = _np(vec.batch.t["pos"]), _np(vec.batch.t["vel"])
        for b, o in enumerate(orc):
            obs_n, node_o, ei_o, dist_o, rew_n, cost_n, done_n, info_n = o.step(list(a[b]))
            assert bool(done[b].all()) == bool(done_n[0]) and bool(done[b].any()) == bool(done[b].all())
            assert np.allclose(rew[b, :, 0], rew_n, rtol=3e-7, atol=2e-6), (t, b)
            check_cost_vs_fp64(cost[b, :, 0], np.array(cost_n, dtype=np.float32), o.get_state()[0], N, (t, b))
            if not done_n[0]:   # bit-exact: the fp32 predicate on the kernel's own positions
                _, c32 = br.reward_cost(ocfg, pos1[b:b + 1], np.float32)
                assert np.array_equal(cost[b, :, 0], c32[0]), (t, b)
            assert [i["cost"] for i in infos[b]] == [float(c) for c in cost[b, :, 0]]
            ep_r[b] += float(np.sum(rew[b, :, 0], dtype=np.float64))   # the episode totals the infos must carry
            ep_c[b] += float(np.sum(cost[b, :, 0], dtype=np.float64))
            if done_n[0]:
                # the episode's totals in the infos, then the worker's reset: the
                # returned observation is the new episode's layout
                for i in infos[b]:
                    assert i["episode"]["r"] == pytest.approx(ep_r[b], rel=1e-5, abs=1e-4)
                    assert i["episode"]["c"] == pytest.approx(ep_c[b], abs=1e-6)
                ep_r[b] = ep_c[b] = 0.0
                obs_n, node_o, ei_o, dist_o = o.reset()
                check_reset_obs(obs[b], obs_n, (t, b))
                resets += 1
            else:
                assert all("episode" not in i for i in infos[b])
                p_o, v_o = o.get_state()
                check_state(pos1[b], p_o, f"vec-env pos t={t} b={b}")
                check_state(vel1[b], v_o, f"vec-env vel t={t} b={b}")
                # observation, node table and graph of the kernel's own positions
                o.set_state(pos1[b].astype(np.float64), vel1[b].astype(np.float64))
                obs_n, node_o, ei_o, dist_o = o._obs()
                check_state(obs[b][:, :4], np.array(obs_n)[:, :4], f"vec-env obs t={t} b={b}")
                assert np.allclose(obs[b][:, 4:], np.array(obs_n)[:, 4:], rtol=0, atol=2.5e-7)
            # node table: every agent sees the env's table
            for i in range(N):
                assert np.array_equal(node[b, i], node[b, 0])
            assert np.array_equal(node[b, 0][:, 6], node_o[:, 6])
            assert np.allclose(node[b, 0][:, :6], node_o[:, :6], rtol=0, atol=2.5e-7)
            # dense adjacency: exactly the oracle's edges, distances within 2 ulp
            want = np.zeros((E, E))
            want[ei_o[0], ei_o[1]] = dist_o
            assert np.array_equal(adj[b, 0] > 0, want > 0), (t, b)
            assert np.allclose(adj[b, 0], want, rtol=2.5e-7, atol=0)
    assert resets == 2 * B        # two auto-resets per env in 12 steps of 5-step episodes
    vec.close()


@pytest.mark.parametrize("N,B", [(6, 32), (24, 16)])
def test_rollout_slots_against_oracle(N, B):
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
    EL, T, seed = 5, 8, 4
    cfg = EnvConfig(n_agents=N, n_envs=B, episode_length=EL, seed=seed)
    ocfg = br.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in br.DEFAULTS})
    env = GpuBatchEnv(cfg, DEV)
    buf = GraphRolloutBuffer(env, episode_length=T)
    g = torch.Generator(device=DEV)
    g.manual_seed(2)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV, generator=g)
    buf.reset(seed=seed)
    buf.capture(acts)
    buf.replay()
    torch.cuda.synchronize()
    assert not bool(buf.overflowed())
    assert torch.equal(buf.actions, acts)
    nf = _np(buf.node_feat)
    E = env.E
    # slot 0: the reset observation (bit-exact layout)
    st0 = br.new_state(ocfg, seed=seed)
    assert np.array_equal(nf[0][:, :, 2:4], st0["pos"])
    step = np.zeros(B, np.int32)
    episode = np.zeros(B, np.int32)
    for t in range(T):
        # the state held in slot t
        pos_t = nf[t][:, :, 2:4].astype(np.float64)
        vel_t = nf[t][:, :N, 0:2].astype(np.float64)
        st = dict(pos=pos_t, vel=vel_t, step=step.copy(), episode=episode.copy(),
                  ep_acc=np.zeros((B, 2)), ep_last=np.zeros((B, 2)))
        nst, ob = br.step(ocfg, st, _np(acts[t]), 1, np.float64, seed=seed)
        done = _np(buf.done[t + 1]).astype(bool)
        assert np.array_equal(done, ob["done"].astype(bool)), t
        assert np.allclose(_np(buf.reward[t + 1]), ob["reward"], rtol=3e-7, atol=2e-6), t
        pos1 = nf[t + 1][:, :, 2:4]
        vel1 = nf[t + 1][:, :N, 0:2]
        keep = ~done
        cost1 = _np(buf.cost[t + 1])
        for b in range(B):
            check_cost_vs_fp64(cost1[b], ob["cost"][b], nst["pos"][b] if keep[b] else
                               br.physics(ocfg, pos_t[b:b + 1], vel_t[b:b + 1], _np(acts[t])[b:b + 1], 1)[0][0],
                               N, (t, b))
        _, c32 = br.reward_cost(ocfg, pos1[keep], np.float32)   # bit-exact on the slot's own positions
        assert np.array_equal(cost1[keep], c32), t
        check_state(pos1[keep], nst["pos"][keep], f"rollout slot {t + 1} pos")
        check_state(vel1[keep], nst["vel"][keep], f"rollout slot {t + 1} vel")
        if done.any():   # re-laid-out envs: the next episode's layout, zero velocity
            lay = br.layout(ocfg, np.nonzero(done)[0], nst["episode"][done], seed)
            assert np.array_equal(pos1[done], lay)
            assert not vel1[done].any()
        # the slot's graph is the fp32 oracle's on the slot's own positions
        ptr, ei, attr = br.edges(ocfg, pos1, np.float32)
        assert np.array_equal(_np(buf.edge_ptr[t + 1]), ptr), t
        n = int(ptr[-1])
        assert np.array_equal(_np(buf.edge_index[t + 1][:, :n]), ei), t
        assert np.allclose(_np(buf.edge_attr[t + 1][:n]), attr, rtol=2.5e-7, atol=0), t
        assert np.array_equal(nf[t + 1], br.node_features(ocfg, pos1, vel1, np.float32)), t
        assert np.array_equal(_np(buf.edge_count[t + 1]), np.diff(ptr).astype(np.int32)), t
        step, episode = nst["step"], nst["episode"]
    # graph_batch of a few samples reproduces the slots' per-env graphs with local ids
    tk = torch.tensor([1, 5, T], dtype=torch.int64)
    bk = torch.tensor([0, B - 1, B // 2], dtype=torch.int64)
    gb = buf.graph_batch(tk, bk)
    for k in range(3):
        t, b = int(tk[k]), int(bk[k])
        ptr = _np(buf.edge_ptr[t])
        e0, e1 = int(ptr[b]), int(ptr[b + 1])
        s0, s1 = int(_np(gb["ptr"])[k]), int(_np(gb["ptr"])[k + 1])
        got = _np(gb["edge_index"][:, s0:s1]) - k * E
        assert np.array_equal(got, _np(buf.edge_index[t][:, e0:e1]).astype(np.int64) - b * E)
    env.close()
