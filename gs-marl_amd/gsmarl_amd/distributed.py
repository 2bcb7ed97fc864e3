"""Multi-GPU sharding of the env batch.

Envs have no cross-dependence, so rank r of W owns the contiguous global env
range [r*B_local, (r+1)*B_local); the Philox layout key uses the *global* env
id (``env_base``), so every env's trajectory is independent of W. The only
collective is the per-episode metric reduction: an ``all_reduce(SUM)`` of a
3-element float64 vector (RCCL over xGMI with backend "nccl"; gloo on CPU).
There is no data-path collective.
"""
from __future__ import annotations

from dataclasses import replace

import torch
import torch.distributed as dist

from .config import EnvConfig


def shard_config(cfg: EnvConfig, rank: int, world_size: int, envs_per_rank: int | None = None) -> EnvConfig:
    """Weak scaling (default): every rank gets ``envs_per_rank`` envs (or
    cfg.n_envs); strong scaling: pass envs_per_rank = total // world_size."""
    n = int(envs_per_rank if envs_per_rank is not None else cfg.n_envs)
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    return replace(cfg, n_envs=n, env_base=int(cfg.env_base) + rank * n)


def all_reduce_metrics(vec: torch.Tensor, group=None, async_op: bool = False):
    """SUM-reduce the per-shard metric vector across ranks (in place). With
    ``async_op`` the collective is only enqueued (RCCL: on its own stream,
    after the work already queued on the current one) and the work handle is
    returned (None without a process group); ``handle.wait()`` orders later
    work after it. Otherwise returns ``vec``."""
    if dist.is_available() and dist.is_initialized():
        work = dist.all_reduce(vec, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        if async_op:
            return work
    return None if async_op else vec


def max_over_ranks(x: float, device="cpu", group=None) -> float:
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
