"""On-device graph rollout buffer — stands in for the reference's
``gsmarl/utils/graph_separated_buffer.py`` (SOURCES.txt:33; SURVEY.md §8(f)
next #2) on the storage side.

The reference copies every step's observations (node features, dense
adjacency, agent ids, rewards, costs, masks) from the env processes into host
NumPy arrays. Here the episode lives in HBM and the env writes each step's
outputs *directly* into the step's slot (``gsm_step_into``: the kernels'
output pointers are redirected, so there is no copy at all), either eagerly
between policy calls or for a whole pre-generated action sequence as one HIP
graph (``gsm_graph_capture_into``).

Storage format for T x B ragged graphs (slot 0 = the observation the episode
starts from, slot t+1 = after action t):

    node_feat  [T+1, B, E, 7] f32          full rows every slot
    reward     [T+1, B, N]    f32          slot t+1: reward of action t
    cost       [T+1, B, N]    f32
    done       [T+1, B]       u8
    edge_count [T+1, B]       i32
    edge_ptr   [T+1, B+1]     i64          CSR offsets into the slot's edges
    edge_index [T+1, 2, cap]  i32          global node ids b*E + e
    edge_attr  [T+1, cap]     f32          distances
    actions    [T, B, N]      i32
    (assign    [T+1, B, N]    i32          ragged scenarios)

``cap`` is per slot (default 8 edges per entity per env, ~6x the mean at the
headline density); a slot whose ``edge_ptr[B]`` exceeds it has its edges
truncated (``overflowed()`` reports it), never written out of bounds.
``graph_batch`` assembles a PyG-style batch of (t, b) samples for the
minibatch generators; ``compute_returns`` is GAE over rewards or costs.
"""
from __future__ import annotations

from typing import Optional

import torch

from .batch import GpuBatchEnv


class GraphRolloutBuffer:
    FIELDS = ("node_feat", "reward", "cost", "done", "edge_count", "edge_ptr", "edge_index", "edge_attr")

    def __init__(self, env: GpuBatchEnv, episode_length: Optional[int] = None,
                 edges_per_env: Optional[int] = None):
        self.env = env
        T = int(episode_length or env.cfg.episode_length)
        B, N, E = env.B, env.N, env.E
        per_env = int(edges_per_env or min(env.sizes.max_edges_per_env, 8 * E))
        cap = B * per_env
        dev = env.device
        f32, i32 = torch.float32, torch.int32
        self.T, self.B, self.N, self.E, self.cap = T, B, N, E, cap
        self.node_feat = torch.zeros(T + 1, B, E, 7, dtype=f32, device=dev)
        self.reward = torch.zeros(T + 1, B, N, dtype=f32, device=dev)
        self.cost = torch.zeros(T + 1, B, N, dtype=f32, device=dev)
        self.done = torch.zeros(T + 1, B, dtype=torch.uint8, device=dev)
        self.edge_count = torch.zeros(T + 1, B, dtype=i32, device=dev)
        self.edge_ptr = torch.zeros(T + 1, B + 1, dtype=torch.int64, device=dev)
        self.edge_index = torch.zeros(T + 1, 2, cap, dtype=i32, device=dev)
        self.edge_attr = torch.zeros(T + 1, cap, dtype=f32, device=dev)
        self.actions = torch.zeros(T, B, N, dtype=i32, device=dev)
        self.ragged = env.cfg.ragged
        if self.ragged:
            self.assign = torch.full((T + 1, B, N), -1, dtype=i32, device=dev)
        self.step = 0

    # ------------------------------------------------------------ storage
    def slot(self, t: int) -> dict:
        """The outputs of slot t as a dict of views (gsm_outputs for the env)."""
        d = {k: getattr(self, k)[t] for k in self.FIELDS}
        if self.ragged:
            d["assign"] = self.assign[t]
        return d

    @property
    def obs(self) -> torch.Tensor:
        """[T+1, B, N, 6] view: the agents' MPE observation (vel, pos, goal-rel)."""
        return self.node_feat[:, :, : self.N, :6]

    @property
    def rewards(self) -> torch.Tensor:
        return self.reward[1:]

    @property
    def costs(self) -> torch.Tensor:
        return self.cost[1:]

    @property
    def masks(self) -> torch.Tensor:
        """[T+1, B, N] f32: 0 after a step that ended the episode (MAPPO masks)."""
        m = 1.0 - self.done.to(torch.float32)
        m[0] = 1.0
        return m.unsqueeze(-1).expand(-1, -1, self.N)

    def overflowed(self) -> torch.Tensor:
        """Device bool: some slot had more edges than the per-slot capacity."""
        return (self.edge_ptr[:, self.B] > self.cap).any()

    # ------------------------------------------------------------ filling
    def reset(self, seed: Optional[int] = None) -> dict:
        """Reset the env and write the first observation into slot 0."""
        self.env.reset(seed=seed, sync_edges=False)
        self.step = 0
        return self.env.observe(out=self.slot(0))

    def insert(self, actions: torch.Tensor) -> dict:
        """env.step(actions) writing straight into the next slot."""
        if self.step >= self.T:
            raise IndexError("buffer is full; call after_update()")
        out = self.env.step(actions, out=self.slot(self.step + 1))
        if actions.dtype == torch.int32:
            self.actions[self.step].copy_(actions)
        elif actions.shape[-1] == 5:          # one-hot: store the index
            self.actions[self.step].copy_(actions.argmax(-1))
        # continuous actions are not stored (the buffer keeps discrete indices)
        self.step += 1
        return out

    def capture(self, actions_seq: torch.Tensor, slot: int = 0) -> None:
        """One HIP graph that steps the whole episode from the env's current
        state, step j writing slot j+1 (actions_seq: int32 [T, B, N])."""
        self.env.capture_into(actions_seq, [self.slot(t + 1) for t in range(self.T)], slot=slot)
        self._graph_actions = actions_seq

    def replay(self, slot: int = 0) -> None:
        """Run a captured episode; slot 0 must already hold its first observation.
        The episode usually runs as one fused rollout launch, whose bounded
        in-launch waits can (in principle) time out and leave invalid edges:
        the next read of the buffer (``graph_batch``, ``validate``) checks."""
        self.env.replay(slot)
        n = self._graph_actions.shape[0]
        idx = torch.arange(self.T, device=self._graph_actions.device) % n
        self.actions.copy_(self._graph_actions[idx])
        self.step = self.T
        self._unchecked = True

    def validate(self) -> None:
        """Raise if a replayed episode's launch gave up a bounded wait (its
        CSR offsets and edges would be wrong). Synchronises; a no-op when no
        replay happened since the last check."""
        if getattr(self, "_unchecked", False):
            self._unchecked = False
            if self.env.roll_gave_up():
                raise RuntimeError("GraphRolloutBuffer: a fused rollout launch gave up waiting on a "
                                   "predecessor workgroup; the episode's edges are invalid")

    def after_update(self) -> None:
        """Carry the last observation into slot 0 for the next rollout."""
        self.validate()
        for k in self.FIELDS + (("assign",) if self.ragged else ()):
            buf = getattr(self, k)
            buf[0].copy_(buf[self.step])
        self.step = 0

    # ------------------------------------------------------------- reading
    def graph_batch(self, t_idx: torch.Tensor, b_idx: torch.Tensor) -> dict:
        """PyG-style batch of K samples (slot t_idx[k], env b_idx[k]): node_feat
        [K*E, 7], edge_index [2, sum] int64 with local ids k*E + e, edge_attr,
        batch [K*E] (sample of each node), ptr [K+1] (edge offsets).
        Raises ValueError if a requested sample's edges were truncated because
        its slot overflowed the per-slot edge capacity (``overflowed()``), and
        RuntimeError if the replayed episode's launch gave up a bounded wait."""
        self.validate()
        E = self.E
        t = t_idx.to(self.edge_ptr.device, torch.int64)
        b = b_idx.to(self.edge_ptr.device, torch.int64)
        K = t.numel()
        start = self.edge_ptr[t, b]
        end = self.edge_ptr[t, b + 1]
        if bool((end > self.cap).any()):
            raise ValueError(f"graph_batch: a requested sample's edges run past the slot capacity {self.cap} "
                             "(the slot overflowed and was truncated); size the buffer with a larger edge "
                             "capacity")
        cnt = end - start
        ptr = torch.zeros(K + 1, dtype=torch.int64, device=t.device)
        torch.cumsum(cnt, 0, out=ptr[1:])
        total = int(ptr[-1].item())
        k = torch.repeat_interleave(torch.arange(K, device=t.device), cnt, output_size=total)
        j = start[k] + (torch.arange(total, device=t.device) - ptr[k])
        tk = t[k]
        src = self.edge_index[tk, 0, j].to(torch.int64)
        dst = self.edge_index[tk, 1, j].to(torch.int64)
        shift = (k - b[k]) * E          # global id b*E + e  ->  local id k*E + e
        return dict(node_feat=self.node_feat[t, b].reshape(K * E, 7),
                    edge_index=torch.stack([src + shift, dst + shift]),
                    edge_attr=self.edge_attr[tk, j],
                    batch=torch.arange(K, device=t.device).repeat_interleave(E),
                    ptr=ptr)

    def render(self, env: int = 0, slots=None, width: int = 700, height: int = 700,
               edges: bool = True) -> torch.Tensor:
        """Frames uint8 [len(slots), H, W, 3] of env ``env`` over the stored
        slots (default: all T+1), straight from the buffer (gsmarl_amd.render);
        ``gsmarl_amd.render.save_gif`` writes them out."""
        from .render import render_frames
        c = self.env.cfg
        slots = range(self.T + 1) if slots is None else slots
        frames = [render_frames(self.node_feat[t], self.edge_ptr[t], self.edge_index[t], [env], width, height,
                                (c.agent_size, c.goal_size, c.obstacle_size), c.world_half or 0.0, edges)
                  for t in slots]
        return torch.cat(frames)

    def compute_returns(self, values: torch.Tensor, gamma: float = 0.99, gae_lambda: float = 0.95,
                        which: str = "reward") -> torch.Tensor:
        """GAE returns [T, B, N] of the rewards (or costs, for the safe-RL
        cost critic) given value predictions values [T+1, B, N]."""
        r = self.rewards if which == "reward" else self.costs
        masks = self.masks
        ret = torch.empty_like(r)
        gae = torch.zeros_like(r[0])
        for t in reversed(range(self.T)):
            delta = r[t] + gamma * values[t + 1] * masks[t + 1] - values[t]
            gae = delta + gamma * gae_lambda * masks[t + 1] * gae
            ret[t] = gae + values[t]
        return ret
