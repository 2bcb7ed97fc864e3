"""GPU-resident vectorised env — stands in for the reference's
``gsmarl/envs/mpe_env/env_wrappers.py`` (SOURCES.txt:11).

The reference (MAPPO / InforMARL lineage) runs ``n_rollout_threads`` env
processes behind ``GraphSubprocVecEnv``: every step pickles actions down a pipe
and observations back. Here all threads are one ``GpuBatchEnv`` on one GPU:
``step`` is two kernel launches and nothing crosses a process boundary. The
surface mirrors the ``ShareVecEnv`` API the runner calls — ``reset()``,
``step_async(actions)`` / ``step_wait()`` / ``step(actions)``, ``close()``,
``num_envs``, ``observation_space`` / ``share_observation_space`` /
``action_space`` (+ ``node_observation_space``, ``adj_observation_space``,
``agent_id_observation_space`` of the graph variant) — with the graph variant's
tuples and the Constrain variants' costs:

    reset() -> obs, agent_id, node_obs, adj
    step(a) -> obs, agent_id, node_obs, adj, rewards, costs, dones, infos

Shapes (MAPPO vec-env convention, B = n_rollout_threads, N agents, E entities):
obs [B,N,6], agent_id [B,N,1], node_obs [B,N,E,7], adj [B,N,E,E],
rewards / costs [B,N,1], dones [B,N] (bool). Episode ends reset in-kernel and
the returned observation is the new episode's, as the MAPPO worker does.

``node_obs="ego"`` gives each agent the node table relative to itself
(InforMARL-style, gsmarl_amd.ego) instead of the shared absolute table.
``output="torch"`` keeps everything on the device (no host copies; node_obs /
adj become expand() views, not copies); ``output="numpy"`` returns host arrays
like the subprocess vec-env. ``graph="dense"`` builds the InforMARL dense
distance adjacency; ``graph="coo"`` returns ``adj=None`` and the batched COO
graph is available from ``graph()`` (edge_index with global node ids,
edge_attr distances, edge_ptr CSR offsets) — the form a PyG-style GNN consumes.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .batch import GpuBatchEnv
from .config import EnvConfig
from .spaces import Box, Discrete


class GpuGraphVecEnv:
    """``GraphSubprocVecEnv`` / ``GraphDummyVecEnv`` replacement on one GPU."""

    def __init__(self, cfg: EnvConfig, device="cuda", output: str = "numpy", graph: str = "dense",
                 node_obs: str = "absolute"):
        if output not in ("numpy", "torch"):
            raise ValueError("output must be 'numpy' or 'torch'")
        if graph not in ("dense", "coo"):
            raise ValueError("graph must be 'dense' or 'coo'")
        if node_obs not in ("absolute", "ego"):
            raise ValueError("node_obs must be 'absolute' or 'ego'")
        self.node_obs = node_obs
        self.cfg = cfg
        self.output = output
        self.graph_mode = graph
        self.batch = GpuBatchEnv(cfg, device)
        self.num_envs = cfg.n_envs
        self.num_agents = cfg.n_agents
        N, E = cfg.n_agents, self.batch.E
        self.action_space = [Discrete(5) for _ in range(N)]
        self.observation_space = [Box(-np.inf, np.inf, (6,)) for _ in range(N)]
        self.share_observation_space = [Box(-np.inf, np.inf, (6 * N,)) for _ in range(N)]
        self.node_observation_space = [Box(-np.inf, np.inf, (E, 7)) for _ in range(N)]
        self.adj_observation_space = [Box(0, np.inf, (E, E)) for _ in range(N)]
        self.agent_id_observation_space = [Box(0, N, (1,)) for _ in range(N)]
        self._pending = None
        self.last = None
        self._agent_id = torch.arange(N, device=self.batch.device, dtype=torch.int64).view(1, N, 1)
        # episode statistics of the envs that finished in the last step
        self.episode_returns = None

    # ------------------------------------------------------------- helpers
    def _actions(self, actions) -> torch.Tensor:
        B, N = self.num_envs, self.num_agents
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions))
        a = a.to(self.batch.device)
        if a.dtype.is_floating_point:
            a = a.to(torch.float32).reshape(B, N, -1)
            if a.shape[-1] not in (5, 2):
                raise ValueError("float actions must be one-hot [B,N,5] or continuous [B,N,2]")
        else:
            a = a.to(torch.int32).reshape(B, N)
        return a.contiguous()

    def _dense_adj(self, out) -> torch.Tensor:
        B, E = self.num_envs, self.batch.E
        adj = torch.zeros(B * E, E, dtype=torch.float32, device=self.batch.device)
        ei = out["edge_index"].to(torch.int64)
        adj[ei[0], ei[1] % E] = out["edge_attr"]
        return adj.view(B, E, E)

    def _host(self, x):
        if x is None or self.output == "torch":
            return x
        return x.cpu().numpy()

    def _graph_obs(self, out):
        B, N = self.num_envs, self.num_agents
        if self.node_obs == "ego":   # agent i's table relative to itself (gsmarl_amd.ego)
            from .ego import EgoView
            node = EgoView(out["node_feat"], N).all()
        else:
            node = out["node_feat"].unsqueeze(1).expand(B, N, *out["node_feat"].shape[1:])
        adj = None
        if self.graph_mode == "dense":
            a = self._dense_adj(out)
            adj = a.unsqueeze(1).expand(B, N, *a.shape[1:])
        aid = self._agent_id.expand(B, N, 1)
        return self._host(out["obs"]), self._host(aid), self._host(node), self._host(adj)

    def _infos(self, out):
        """Per env, per agent dicts with the agent's cost; finished envs also
        carry the finished episode's totals (sum reward, sum cost), degenerate
        envs their App. A S16 flags."""
        c = out["cost"].cpu().numpy()
        d = out["done"].cpu().numpy().astype(bool)
        deg = out["degenerate"].cpu().numpy()
        last = self.batch.t["ep_last"].cpu().numpy() if d.any() else None
        infos = []
        for b in range(self.num_envs):
            row = [{"cost": float(c[b, i])} for i in range(self.num_agents)]
            if deg[b]:   # App. A S16 flags (coincident colliders / non-finite agent)
                for info in row:
                    info["degenerate"] = int(deg[b])
            if d[b]:
                for info in row:
                    info["episode"] = {"r": float(last[b, 0]), "c": float(last[b, 1])}
            infos.append(row)
        return infos

    # ---------------------------------------------------------------- API
    def reset(self, seed: Optional[int] = None, env_mask=None):
        """Reset every env (or those with env_mask != 0); returns
        (obs, agent_id, node_obs, adj) of the whole batch."""
        out = self.batch.reset(seed=seed, env_mask=env_mask, sync_edges=self.graph_mode == "dense")
        self.last = out
        return self._graph_obs(out)

    def step_async(self, actions):
        self._pending = self._actions(actions)

    def step_wait(self):
        if self._pending is None:
            raise RuntimeError("step_wait() without step_async()")
        out = self.batch.step(self._pending, sync_edges=self.graph_mode == "dense")
        self._pending = None
        self.last = out
        obs, aid, node, adj = self._graph_obs(out)
        rew = out["reward"].unsqueeze(-1)
        cost = out["cost"].unsqueeze(-1)
        done = out["done"].bool().unsqueeze(1).expand(self.num_envs, self.num_agents)
        infos = self._infos(out) if self.output == "numpy" else None
        return obs, aid, node, adj, self._host(rew), self._host(cost), self._host(done), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def graph(self):
        """Batched COO graph of the latest observation (device tensors)."""
        o = self.last if self.last is not None else self.batch.outputs()
        return dict(node_feat=o["node_feat"].reshape(-1, 7), edge_index=o["edge_index"],
                    edge_attr=o["edge_attr"], edge_ptr=o["edge_ptr"])

    def episode_metrics(self) -> torch.Tensor:
        return self.batch.episode_metrics()

    def close(self):
        self.batch.close()


def make_train_env(all_args, device="cuda", output: str = "numpy", graph: str = "dense"):
    """MAPPO-style factory: ``all_args`` carries ``scenario_name``,
    ``num_agents``, ``n_rollout_threads``, ``seed``, ``episode_length`` (and
    optionally ``num_obstacles``, ``env_base``), as the reference's
    train_mpe.py args do. Thread r's env has global id env_base + r."""
    from .make_env import SCENARIO_ALIASES
    kw = dict(scenario=SCENARIO_ALIASES[getattr(all_args, "scenario_name", "navigation")],
              n_agents=int(all_args.num_agents), n_envs=int(all_args.n_rollout_threads),
              seed=int(getattr(all_args, "seed", 0)),
              episode_length=int(getattr(all_args, "episode_length", 100)),
              env_base=int(getattr(all_args, "env_base", 0)))
    if getattr(all_args, "num_obstacles", None) is not None:
        kw["n_obstacles"] = int(all_args.num_obstacles)
    return GpuGraphVecEnv(EnvConfig(**kw), device=device, output=output, graph=graph)


def make_eval_env(all_args, device="cuda", output: str = "numpy", graph: str = "dense"):
    """Evaluation envs: ``n_eval_rollout_threads`` of them, seeded apart from
    training (seed * 50000, the MAPPO convention), ids after the training envs."""
    import copy
    a = copy.copy(all_args)
    a.n_rollout_threads = int(getattr(all_args, "n_eval_rollout_threads", 1))
    a.seed = int(getattr(all_args, "seed", 0)) * 50000
    a.env_base = int(getattr(all_args, "n_rollout_threads", 0))
    return make_train_env(a, device=device, output=output, graph=graph)
