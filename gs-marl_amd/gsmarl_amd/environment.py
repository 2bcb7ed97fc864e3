"""Drop-in surface for ``gsmarl/envs/mpe_env/multiagent/environment.py``
(SOURCES.txt:15). The reference defines three env classes (readme.md:29-41):

* ``MultiAgentEnv``              fixed-size obs, no cost          (readme.md:29-33)
* ``MultiAgentConstrainEnv``     fixed-size obs + per-agent cost  (readme.md:34-37)
* ``MultiAgentGraphConstrainEnv`` variable-size graph obs + cost  (readme.md:38-41)

Same names, same ``reset()`` / ``step(action_n)`` methods. Return conventions
(the reference's exact tuples are not published): MPE/MAPPO
``(obs_n, reward_n, done_n, info_n)``; the Constrain variants insert
``cost_n`` after ``reward_n`` and mirror it as ``info_n[i]['cost']``; the
graph variant follows InforMARL ``(obs_n, agent_id_n, node_obs_n, adj_n, ...)``.

With ``n_envs == 1`` the values are per-agent lists of numpy arrays exactly as
a single MPE env returns them (ragged scenarios: the env's own N_env agents;
actions for N_env agents are padded with no-ops). With ``n_envs > 1`` they are stacked numpy
arrays in the MAPPO vec-env shapes (obs [B,N,6], reward [B,N,1], done [B,N]).
Either way ``self.last`` keeps the device tensors of the latest call, and
``graph()`` returns the batched COO graph without building dense adjacency.
Every call runs the HIP step path (GpuBatchEnv); there is no CPU fallback.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .batch import GpuBatchEnv
from .config import EnvConfig
from .spaces import Box, Discrete


class MultiAgentEnv:
    with_cost = False
    with_graph = False

    def __init__(self, cfg: Optional[EnvConfig] = None, device="cuda", **kw):
        self.cfg = cfg if cfg is not None else EnvConfig(**kw)
        self.batch = GpuBatchEnv(self.cfg, device)
        self.n = self.cfg.n_agents
        self.num_envs = self.cfg.n_envs
        self.world_length = self.cfg.episode_length
        self.current_step = 0
        self.action_space = [Discrete(5) for _ in range(self.n)]
        self.observation_space = [Box(-np.inf, np.inf, (6,)) for _ in range(self.n)]
        self.share_observation_space = [Box(-np.inf, np.inf, (6 * self.n,)) for _ in range(self.n)]
        E = self.batch.E
        self.node_observation_space = [Box(-np.inf, np.inf, (E, 7)) for _ in range(self.n)]
        self.adj_observation_space = [Box(0, np.inf, (E, E)) for _ in range(self.n)]
        self.agent_id_observation_space = [Box(0, self.n, (1,)) for _ in range(self.n)]
        self.last = None
        self.n_active = self.n   # ragged single env: its N_env after reset

    def _refresh_active(self, out):
        if self.cfg.ragged and self.num_envs == 1:
            self.n_active = int(out["n_agents_env"][0].item())

    # ---------------------------------------------------------------- actions
    def _to_actions(self, action_n) -> torch.Tensor:
        dev, B, N = self.batch.device, self.num_envs, self.n
        if isinstance(action_n, torch.Tensor):
            a = action_n.to(dev)
        else:
            a = torch.as_tensor(np.asarray(action_n), device=dev)
        if a.dtype.is_floating_point:
            a = a.to(torch.float32)
            if a.dim() == 2 and B == 1:
                a = a.unsqueeze(0)
            if a.dim() == 3 and a.shape[-1] not in (5, 2):
                raise ValueError("float actions must be one-hot [.., 5] or continuous [.., 2]")
        else:
            a = a.to(torch.int32)
            if a.dim() == 1 and B == 1:
                a = a.unsqueeze(0)
            if a.dim() == 3 and a.shape[-1] == 1:
                a = a[..., 0]
        if B == 1 and a.dim() >= 2 and a.shape[0] == 1 and a.shape[1] < N:   # ragged env: pad with no-ops
            pad = torch.zeros((1, N - a.shape[1], *a.shape[2:]), dtype=a.dtype, device=dev)
            a = torch.cat([a, pad], dim=1)
        return a.reshape(B, N, *a.shape[2:]).contiguous()

    # --------------------------------------------------------------- outputs
    def _per_agent(self, x: np.ndarray):
        """[B, N, ...] -> per-agent list (n_envs == 1) or the stacked array."""
        if self.num_envs == 1:
            return [x[0, i] for i in range(self.n_active)]
        return x

    def _obs(self, out):
        return self._per_agent(out["obs"].cpu().numpy())

    def _reward(self, out):
        r = out["reward"].cpu().numpy()
        if self.num_envs == 1:
            return [float(v) for v in r[0, : self.n_active]]
        return r[..., None]

    def _cost(self, out):
        c = out["cost"].cpu().numpy()
        if self.num_envs == 1:
            return [float(v) for v in c[0, : self.n_active]]
        return c[..., None]

    def _done(self, out):
        d = out["done"].cpu().numpy().astype(bool)
        if self.num_envs == 1:
            return [bool(d[0])] * self.n_active
        return np.repeat(d[:, None], self.n, axis=1)

    def _info(self, out, cost=None):
        """Per-agent info dicts: the cost (Constrain variants) and, when the
        env is in a degenerate state (App. A S16: coincident colliders, or a
        non-finite agent under strict_degenerate), ``degenerate`` = its flags."""
        deg = out["degenerate"].cpu().numpy()
        if self.num_envs == 1:
            infos = [{} for _ in range(self.n_active)]
            if cost is not None:
                for i, c in enumerate(cost):
                    infos[i]["cost"] = c
            if deg[0]:
                for info in infos:
                    info["degenerate"] = int(deg[0])
            return infos
        infos = [[{} for _ in range(self.n)] for _ in range(self.num_envs)]
        for b in range(self.num_envs):
            for i in range(self.n):
                if cost is not None:
                    infos[b][i]["cost"] = float(cost[b, i, 0])
                if deg[b]:
                    infos[b][i]["degenerate"] = int(deg[b])
        return infos

    # ------------------------------------------------------------------- API
    def reset(self, seed: Optional[int] = None):
        out = self.batch.reset(seed=seed, sync_edges=self.with_graph)
        self.current_step = 0
        self.last = out
        self._refresh_active(out)
        return self._obs(out)

    def step(self, action_n):
        out = self.batch.step(self._to_actions(action_n), sync_edges=self.with_graph)
        self.current_step += 1
        self.last = out
        return self._obs(out), self._reward(out), self._done(out), self._info(out)

    def graph(self):
        """Batched COO graph of the latest observation (device tensors)."""
        o = self.last if self.last is not None else self.batch.outputs()
        return dict(node_feat=o["node_feat"].reshape(-1, 7), edge_index=o["edge_index"],
                    edge_attr=o["edge_attr"], edge_ptr=o["edge_ptr"])

    def render(self, mode: str = "rgb_array", env_ids=(0,), width: int = 700, height: int = 700,
               edges: bool = True):
        """MPE ``render``: one RGB frame (uint8 [H, W, 3] NumPy array) per env
        of ``env_ids``, drawn on the GPU from the current node features and
        edges (gsmarl_amd.render). Only ``rgb_array`` (there is no display)."""
        if mode != "rgb_array":
            raise NotImplementedError("only mode='rgb_array' (no window system)")
        frames = self.batch.render(env_ids, width=width, height=height, edges=edges)
        return list(frames.cpu().numpy())

    def close(self):
        self.batch.close()


class MultiAgentConstrainEnv(MultiAgentEnv):
    with_cost = True

    def step(self, action_n):
        out = self.batch.step(self._to_actions(action_n), sync_edges=self.with_graph)
        self.current_step += 1
        self.last = out
        cost = self._cost(out)
        return (self._obs(out), self._reward(out), cost, self._done(out), self._info(out, cost))


class MultiAgentGraphConstrainEnv(MultiAgentConstrainEnv):
    """node_obs="absolute" (default): every agent receives the env's node
    table; node_obs="ego": agent i receives it relative to itself
    (InforMARL-style, gsmarl_amd.ego), derived on the device per call."""
    with_graph = True

    def __init__(self, cfg: Optional[EnvConfig] = None, device="cuda", node_obs: str = "absolute", **kw):
        if node_obs not in ("absolute", "ego"):
            raise ValueError("node_obs must be 'absolute' or 'ego'")
        super().__init__(cfg, device, **kw)
        self.node_obs = node_obs

    def _dense_adj(self, out) -> np.ndarray:
        """InforMARL-style adjacency: adj[b, s, d] = distance of edge s->d, else 0."""
        B, E = self.num_envs, self.batch.E
        adj = torch.zeros(B * E, E, dtype=torch.float32, device=self.batch.device)
        ei = out["edge_index"].to(torch.int64)
        adj[ei[0], ei[1] % E] = out["edge_attr"]
        return adj.view(B, E, E).cpu().numpy()

    def _graph_obs(self, out):
        adj = self._dense_adj(out)
        aid = out["agent_id"].cpu().numpy()[..., None]
        B, N = self.num_envs, self.n
        if self.node_obs == "ego":
            from .ego import EgoView
            node = EgoView(out["node_feat"], N).all().cpu().numpy()            # [B, N, E, 7]
            if self.num_envs == 1:
                n = self.n_active
                return ([aid[0, i] for i in range(n)], [node[0, i] for i in range(n)], [adj[0]] * n)
            return (aid, node, np.repeat(adj[:, None], N, axis=1))
        node = out["node_feat"].cpu().numpy()
        if self.num_envs == 1:
            n = self.n_active
            return ([aid[0, i] for i in range(n)], [node[0]] * n, [adj[0]] * n)
        return (aid, np.repeat(node[:, None], N, axis=1), np.repeat(adj[:, None], N, axis=1))

    def reset(self, seed: Optional[int] = None):
        obs = super().reset(seed)
        aid, node, adj = self._graph_obs(self.last)
        return obs, aid, node, adj

    def step(self, action_n):
        obs, rew, cost, done, info = super().step(action_n)
        aid, node, adj = self._graph_obs(self.last)
        return obs, aid, node, adj, rew, cost, done, info
