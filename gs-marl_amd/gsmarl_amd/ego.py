"""Ego-relative node features (InforMARL lineage, SURVEY.md a7 [EXT]).

The env kernels write ONE absolute node-feature table per env
([B, E, 7]: vx vy px py gx-px gy-py type). InforMARL-style graph envs hand
each agent i its own view of that table, relative to itself. Here that view
is derived on demand from the absolute table on the device — nothing N-fold
is written by the step path — by ``EgoView`` (agent i's [B, E, 7] slice on
indexing, the full [B, N, E, 7] only when asked).

Row e of agent i's view [DECISION: InforMARL's relative features; parity
unpinned — the reference's graph env is absent, readme.md:1]:

    [ v_e - v_i,  p_e - p_i,  (g_e - p_e) + (p_e - p_i),  type_e ]

with the goal term (agent e's own goal or assigned slot, relative to ego
agent i) only for agent rows (type 0); 0 for goals, obstacles and padding.
Velocities of immovable entities are 0 in the table, so their relative
velocity is -v_i.
"""
from __future__ import annotations

import torch


def ego_rows(node_feat: torch.Tensor, agent: int | torch.Tensor) -> torch.Tensor:
    """Agent ``agent``'s view [B, E, 7] of node_feat [B, E, 7] (a scalar
    index or a [B] tensor of per-env agent indices)."""
    B = node_feat.shape[0]
    if isinstance(agent, torch.Tensor):
        ego = node_feat[torch.arange(B, device=node_feat.device), agent.to(node_feat.device)]   # [B, 7]
    else:
        ego = node_feat[:, int(agent)]
    return _relative(node_feat, ego[:, None, :])


def _relative(nf: torch.Tensor, ego: torch.Tensor) -> torch.Tensor:
    vel, pos, grel, typ = nf[..., 0:2], nf[..., 2:4], nf[..., 4:6], nf[..., 6:7]
    dv = vel - ego[..., 0:2]
    dp = pos - ego[..., 2:4]
    is_agent = (typ == 0).to(nf.dtype)
    dg = (grel + dp) * is_agent
    return torch.cat([dv, dp, dg, typ.expand_as(dv[..., :1])], dim=-1)


class EgoView:
    """Lazy per-agent view of a [B, E, 7] node table: ``view[i]`` is agent
    i's [B, E, 7] relative table, ``view.all()`` the [B, N, E, 7] stack."""

    def __init__(self, node_feat: torch.Tensor, n_agents: int):
        self.node_feat = node_feat
        self.n_agents = int(n_agents)

    def __len__(self) -> int:
        return self.n_agents

    def __getitem__(self, i: int) -> torch.Tensor:
        if not 0 <= int(i) < self.n_agents:
            raise IndexError(i)
        return ego_rows(self.node_feat, int(i))

    def all(self) -> torch.Tensor:
        nf = self.node_feat                               # [B, E, 7]
        ego = nf[:, : self.n_agents]                      # [B, N, 7]
        return _relative(nf[:, None, :, :], ego[:, :, None, :])
