"""GPU-resident vectorised env — stands in for the reference's
``gsmarl/envs/mpe_env/env_wrappers.py`` (SOURCES.txt:11).

The reference (MAPPO / InforMARL lineage) runs ``n_rollout_threads`` env
processes behind ``GraphSubprocVecEnv``: every step pickles actions down a pipe
and observations back. Here all threads are one ``GpuBatchEnv`` on one GPU:
``step`` is one kernel launch (the one-launch step of the navigation shapes;
the step + emit pair elsewhere) and nothing crosses a process boundary. The
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
like the subprocess vec-env — the per-env tables cross PCIe once and the
per-agent axis is a read-only ``np.broadcast_to`` view of them (at 24 agents x
8192 envs a materialised dense ``adj`` would be 4.1 GB per step, the view costs
the 170 MB table), and ``infos`` is a lazy list (``LazyInfos``: the per-agent
dicts are built when an env's entry is read). ``graph="dense"`` builds the InforMARL dense
distance adjacency; ``graph="coo"`` returns ``adj=None`` and the batched COO
graph is available from ``graph()`` (edge_index with global node ids,
edge_attr distances, edge_ptr CSR offsets) — the form a PyG-style GNN consumes.
"""
from __future__ import annotations

import warnings
from collections.abc import Sequence
from typing import Optional

import numpy as np
import torch

from .batch import GpuBatchEnv
from .config import EnvConfig
from .spaces import Box, Discrete


# host bytes per step above which output="numpy", graph="dense" warns at
# construction (the [B, E, E] dense adjacency table that crosses PCIe)
DENSE_HOST_WARN_BYTES = 256 << 20


class LazyInfos(Sequence):
    """The vec-env's ``infos``: a list of B per-env lists of N per-agent dicts
    ({"cost"}, finished envs also {"episode": {"r", "c"}}, degenerate envs
    {"degenerate"}), built when an env's entry is read instead of 196,608
    dicts per step at the headline size. The step's costs, done flags,
    degenerate flags and finished-episode totals come over in one host copy
    each; ``finished`` (env indices) and ``episode_stats`` ([n, 2]: sum reward,
    sum cost) give the finished episodes without building any dict."""

    def __init__(self, cost: np.ndarray, done: np.ndarray, deg: np.ndarray, last: Optional[np.ndarray]):
        self._cost, self._done, self._deg, self._last = cost, done, deg, last
        self.finished = np.flatnonzero(done)
        self.episode_stats = last[self.finished] if last is not None else np.zeros((0, 2), np.float32)

    def __len__(self):
        return self._cost.shape[0]

    def _env(self, b):
        row = [{"cost": float(c)} for c in self._cost[b]]
        if self._deg[b]:   # App. A S16 flags (coincident colliders / non-finite agent)
            for info in row:
                info["degenerate"] = int(self._deg[b])
        if self._done[b]:
            ep = {"r": float(self._last[b, 0]), "c": float(self._last[b, 1])}
            for info in row:
                info["episode"] = dict(ep)
        return row

    def __getitem__(self, b):
        if isinstance(b, slice):
            return [self._env(i) for i in range(*b.indices(len(self)))]
        b = int(b)
        if b < 0:
            b += len(self)
        if not 0 <= b < len(self):
            raise IndexError(b)
        return self._env(b)


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
        if output == "numpy" and graph == "dense":
            B = cfg.n_envs
            host = B * E * E * 4 + B * E * 7 * 4
            if host > DENSE_HOST_WARN_BYTES:
                warnings.warn(f"GpuGraphVecEnv(output='numpy', graph='dense') at {B} envs x {E} entities moves "
                              f"{host / 2**20:.0f} MB to the host every step (the dense adjacency table); "
                              "graph='coo' or output='torch' keep the graph on the device", stacklevel=2)

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

    def _per_agent(self, table):
        """[B, ...] per-env table -> [B, N, ...] per agent: an expand() view on
        the device, a read-only np.broadcast_to view of ONE host copy of the
        table in numpy mode (the per-agent copies are never materialised)."""
        B, N = self.num_envs, self.num_agents
        if self.output == "torch":
            return table.unsqueeze(1).expand(B, N, *table.shape[1:])
        h = table.cpu().numpy()
        return np.broadcast_to(h[:, None], (B, N) + h.shape[1:])

    def _graph_obs(self, out):
        B, N = self.num_envs, self.num_agents
        if self.node_obs == "ego":   # agent i's table relative to itself (gsmarl_amd.ego)
            from .ego import EgoView
            node = self._host(EgoView(out["node_feat"], N).all())
        else:
            node = self._per_agent(out["node_feat"])
        adj = self._per_agent(self._dense_adj(out)) if self.graph_mode == "dense" else None
        aid = self._agent_id.expand(B, N, 1)
        if self.output == "numpy":
            aid = np.broadcast_to(np.arange(N, dtype=np.int64).reshape(1, N, 1), (B, N, 1))
        return self._host(out["obs"]), aid, node, adj

    def _infos(self, out):
        """Per env, per agent dicts with the agent's cost; finished envs also
        carry the finished episode's totals (sum reward, sum cost), degenerate
        envs their App. A S16 flags — as a LazyInfos list."""
        d = out["done"].cpu().numpy().astype(bool)
        last = self.batch.t["ep_last"].cpu().numpy() if d.any() else None
        return LazyInfos(out["cost"].cpu().numpy(), d, out["degenerate"].cpu().numpy(), last)

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
        # (u8 0/1 reinterpreted as bool: a view, no conversion kernel)
        done = out["done"].view(torch.bool).unsqueeze(1).expand(self.num_envs, self.num_agents)
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
