"""GPU-resident vec-env (gsmarl_amd.vec_env) against
the batch API it wraps and the MAPPO vec-env contract (shapes, auto-reset,
per-agent cost infos, episode totals)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _args(**kw):
    a = dict(scenario_name="navigation", num_agents=4, n_rollout_threads=16, seed=3, episode_length=5,
             n_eval_rollout_threads=2)
    a.update(kw)
    return SimpleNamespace(**a)


def test_shapes_and_contract():
    from gsmarl_amd import make_train_env
    envs = make_train_env(_args(), device=DEV)
    B, N, E = 16, 4, 12
    obs, aid, node, adj = envs.reset(seed=3)
    assert obs.shape == (B, N, 6) and aid.shape == (B, N, 1) and node.shape == (B, N, E, 7)
    assert adj.shape == (B, N, E, E)
    assert np.array_equal(aid[0, :, 0], np.arange(N))
    acts = np.random.default_rng(0).integers(0, 5, size=(B, N, 1))
    for t in range(5):
        obs, aid, node, adj, rew, cost, done, infos = envs.step(acts)
    assert rew.shape == (B, N, 1) and cost.shape == (B, N, 1) and done.shape == (B, N)
    assert done.all()                      # episode_length 5: every env finished at t = 4
    assert len(infos) == B and len(infos[0]) == N and "episode" in infos[0][0]
    assert infos[3][2]["cost"] == float(cost[3, 2, 0])
    # the returned observation is the new episode's (in-kernel auto-reset)
    assert np.all(envs.batch.t["step_count"].cpu().numpy() == 0)
    envs.close()


def test_matches_batch_env_and_dense_adj():
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GpuGraphVecEnv
    cfg = dict(n_agents=6, n_envs=32, seed=9)
    vec = GpuGraphVecEnv(EnvConfig(**cfg), DEV, output="torch")
    ref = GpuBatchEnv(EnvConfig(**cfg), DEV)
    vec.reset(seed=9)
    ref.reset(seed=9)
    a = torch.randint(0, 5, (32, 6), dtype=torch.int32, device=DEV)
    obs, aid, node, adj, rew, cost, done, _ = vec.step(a)
    out = ref.step(a)
    assert torch.equal(obs, out["obs"]) and torch.equal(rew[..., 0], out["reward"])
    assert torch.equal(node[:, 3], out["node_feat"]) and torch.equal(cost[..., 0], out["cost"])
    ei = out["edge_index"].long()
    E = ref.E
    assert torch.allclose(adj[ei[0] // E, 0, ei[0] % E, ei[1] % E], out["edge_attr"])
    assert int((adj[:, 0] > 0).sum()) <= ei.shape[1]
    vec.close()
    ref.close()


def test_coo_mode_and_partial_reset():
    from gsmarl_amd import make_train_env
    envs = make_train_env(_args(n_rollout_threads=8, episode_length=100), device=DEV, output="torch", graph="coo")
    envs.reset(seed=1)
    for _ in range(3):
        obs, aid, node, adj, rew, cost, done, infos = envs.step(torch.zeros(8, 4, dtype=torch.int32))
    assert adj is None and infos is None
    g = envs.graph()
    assert g["edge_index"].shape[0] == 2 and g["edge_ptr"].shape == (9,)
    mask = torch.zeros(8, dtype=torch.uint8)
    mask[2] = 1
    envs.reset(env_mask=mask)
    sc = envs.batch.t["step_count"].cpu().numpy()
    assert sc[2] == 0 and np.all(np.delete(sc, 2) == 3)
    envs.close()


def test_eval_env_ids_follow_training_envs():
    from gsmarl_amd import make_eval_env
    ev = make_eval_env(_args(), device=DEV)
    assert ev.num_envs == 2 and ev.cfg.env_base == 16 and ev.cfg.seed == 3 * 50000
    ev.close()


def test_ego_node_obs():
    """node_obs="ego" (InforMARL-style per-agent view, gsmarl_amd.ego): agent
    i's table is the absolute table relative to agent i, in the vec-env and in
    the single-env drop-in class."""
    from gsmarl_amd import EnvConfig, GpuGraphVecEnv, MultiAgentGraphConstrainEnv
    from gsmarl_amd.ego import EgoView
    cfg = dict(n_agents=5, n_envs=8, seed=4)
    vec = GpuGraphVecEnv(EnvConfig(**cfg), DEV, output="torch", node_obs="ego")
    vec.reset(seed=4)
    a = torch.randint(0, 5, (8, 5), dtype=torch.int32, device=DEV)
    obs, aid, node, adj, rew, cost, done, _ = vec.step(a)
    nf = vec.batch.t["node_feat"]
    assert node.shape == (8, 5, nf.shape[1], 7)
    assert torch.equal(node, EgoView(nf, 5).all())
    for i in range(5):
        assert torch.all(node[:, i, i, 0:4] == 0)
        assert torch.allclose(node[:, i, :, 2:4], nf[:, :, 2:4] - nf[:, i:i + 1, 2:4])
    vec.close()
    env = MultiAgentGraphConstrainEnv(EnvConfig(n_agents=4, n_envs=1, seed=2), DEV, node_obs="ego")
    obs_n, aid_n, node_n, adj_n = env.reset(seed=2)
    nf = env.batch.t["node_feat"]
    assert len(node_n) == 4
    for i in range(4):
        assert np.array_equal(node_n[i], EgoView(nf, 4)[i][0].cpu().numpy())
    env.close()


def test_numpy_mode_broadcast_views_and_lazy_infos():
    """output="numpy": node_obs / adj / agent_id are read-only broadcast views
    of one host copy of each per-env table (no per-agent copies), equal to the
    torch mode's expand() views; infos is a LazyInfos list whose entries and
    finished-episode totals match the step's costs and ep_last."""
    from gsmarl_amd import make_train_env
    from gsmarl_amd.vec_env import LazyInfos
    kw = dict(n_rollout_threads=64, num_agents=6, episode_length=3)
    envs = make_train_env(_args(**kw), device=DEV)
    tenv = make_train_env(_args(**kw), device=DEV, output="torch")
    envs.reset(seed=5)
    tenv.reset(seed=5)
    acts = np.random.default_rng(1).integers(0, 5, size=(3, 64, 6)).astype(np.int32)
    for t in range(3):
        obs, aid, node, adj, rew, cost, done, infos = envs.step(acts[t])
        tob, taid, tnode, tadj, *_ = tenv.step(acts[t])
    assert node.strides[1] == 0 and adj.strides[1] == 0 and aid.strides[0] == 0
    assert not node.flags.writeable
    assert np.array_equal(node, tnode.cpu().numpy()) and np.array_equal(adj, tadj.cpu().numpy())
    assert np.array_equal(aid, taid.cpu().numpy()) and np.array_equal(obs, tob.cpu().numpy())
    assert isinstance(infos, LazyInfos) and len(infos) == 64
    assert np.array_equal(infos.finished, np.arange(64))          # episode_length 3: all finished
    last = envs.batch.t["ep_last"].cpu().numpy()
    assert np.array_equal(infos.episode_stats, last)
    assert infos[5][2]["cost"] == float(cost[5, 2, 0])
    assert infos[-1][0]["episode"] == {"r": float(last[63, 0]), "c": float(last[63, 1])}
    assert len(infos[10:13]) == 3 and len(list(iter(infos))) == 64
    envs.close()
    tenv.close()


def test_dense_numpy_mode_warns_at_headline_size():
    """output="numpy", graph="dense" past 256 MB of host tables per step warns
    at construction (24 agents x 8192 envs: 170 MB of adjacency + 16 MB of node
    features per step stays under it; 96 agents x 1024 envs: 340 MB warns)."""
    import warnings as w
    from gsmarl_amd import EnvConfig, GpuGraphVecEnv
    with w.catch_warnings():
        w.simplefilter("error")
        GpuGraphVecEnv(EnvConfig(n_agents=24, n_envs=8192), DEV).close()
    with pytest.warns(UserWarning, match="graph='coo'"):
        GpuGraphVecEnv(EnvConfig(n_agents=96, n_envs=1024), DEV).close()
