"""GNN message passing over the env graph.

The reference's actor/critic encode the graph observation with a GNN
(gsmarl/algorithms, SOURCES.txt:8; torch-geometric 2.3.1, requirements.txt:119;
the InforMARL lineage uses ``TransformerConv`` with the edge distance as a
1-d edge feature). torch-geometric is not available here, so this module
restates that layer:

* projections ``q/k/v/skip = x @ W + b`` and the edge projection ``w_e`` are
  dense GEMMs (torch.matmul -> hipBLASLt / MFMA);
* the graph part — per-edge scores, segmented softmax over each target's
  neighbours, weighted aggregation — is the HIP kernel behind
  ``gsm_attn_aggregate`` (gsm_gnn.hip) on the rollout / inference path, and the
  equivalent torch formulation (``attn_aggregate_ref``) where gradients are
  needed (training) or as the numerics reference.

Graph format: CSR over targets (``row_ptr`` [n+1] int64, ``col`` int32
sources, ``edge_w`` per CSR entry). The env graphs are symmetric (every radius
edge and agent<->goal edge is emitted both ways), so the row-major COO the
env emits *is* that CSR: ``env_csr`` only adds per-node row offsets.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import torch

from . import _lib


def env_csr(edge_index: torch.Tensor, n_nodes: int) -> torch.Tensor:
    """Per-node row offsets [n_nodes+1] (int64) of a row-major edge list whose
    sources are sorted (the env's COO output)."""
    cnt = torch.bincount(edge_index[0].to(torch.int64), minlength=n_nodes)
    ptr = torch.zeros(n_nodes + 1, dtype=torch.int64, device=edge_index.device)
    torch.cumsum(cnt, 0, out=ptr[1:])
    return ptr


def attn_aggregate_ref(q, k, v, row_ptr, col, edge_w=None, w_e=None, skip=None, heads=1, scale=None):
    """Torch (differentiable) formulation of gsm_attn_aggregate."""
    n, HC = q.shape
    Cc = HC // heads
    scale = 1.0 / math.sqrt(Cc) if scale is None else scale
    deg = row_ptr[1:] - row_ptr[:-1]
    tgt = torch.repeat_interleave(torch.arange(n, device=q.device), deg, output_size=col.numel())
    src = col.to(torch.int64)
    e = 0.0
    if edge_w is not None:
        e = edge_w[:, None] * w_e[None, :]
    kj = (k[src] + e).view(-1, heads, Cc)
    vj = (v[src] + e).view(-1, heads, Cc)
    s = (q[tgt].view(-1, heads, Cc) * kj).sum(-1) * scale                     # [nE, H]
    smax = torch.full((n, heads), -math.inf, device=q.device, dtype=q.dtype)
    smax = smax.scatter_reduce(0, tgt[:, None].expand(-1, heads), s, reduce="amax", include_self=True)
    a = torch.exp(s - smax[tgt])
    den = torch.zeros(n, heads, device=q.device, dtype=q.dtype).index_add(0, tgt, a)
    alpha = a / den[tgt]
    out = torch.zeros(n, heads, Cc, device=q.device, dtype=q.dtype).index_add(0, tgt, alpha[..., None] * vj)
    out = out.view(n, HC)
    if skip is not None:
        out = out + skip
    return out


def attn_aggregate(q, k, v, row_ptr, col, edge_w=None, w_e=None, skip=None, heads=1, scale=None):
    """HIP kernel (no autograd): see gsm_attn_aggregate in include/gsm.h."""
    n, HC = q.shape
    Cc = HC // heads
    scale = 1.0 / math.sqrt(Cc) if scale is None else float(scale)
    dev = q.device
    if dev.type != "cuda":
        raise _lib.GsmError("attn_aggregate needs a ROCm GPU; use attn_aggregate_ref on the CPU")
    for name, t, dt in (("q", q, torch.float32), ("k", k, torch.float32), ("v", v, torch.float32),
                        ("row_ptr", row_ptr, torch.int64), ("col", col, torch.int32)):
        if t.dtype != dt or not t.is_contiguous() or t.device != dev:
            raise ValueError(f"{name}: need a contiguous {dt} tensor on {dev}")
    if edge_w is not None and (edge_w.dtype != torch.float32 or w_e is None):
        raise ValueError("edge_w: float32, with w_e")
    lib = _lib.load()
    out = torch.empty_like(q)

    def ptr(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rc = lib.gsm_attn_aggregate(ptr(q), ptr(k), ptr(v), ptr(edge_w), ptr(w_e.contiguous() if w_e is not None else None),
                                ptr(row_ptr), ptr(col), ptr(skip.contiguous() if skip is not None else None),
                                int(n), int(heads), int(Cc), scale, ptr(out), stream)
    _lib.check(lib, rc, None, "gsm_attn_aggregate")
    return out


class TransformerConv(torch.nn.Module):
    """``TransformerConv(in_channels, out_channels, heads, concat, edge_dim=1,
    root_weight=True)`` in the torch-geometric parameterisation, with the
    aggregation on the HIP kernel when no gradient is needed."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 edge_dim: Optional[int] = 1, root_weight: bool = True, use_kernel: bool = True):
        super().__init__()
        self.heads, self.out_channels, self.concat = heads, out_channels, concat
        HC = heads * out_channels
        self.lin_query = torch.nn.Linear(in_channels, HC)
        self.lin_key = torch.nn.Linear(in_channels, HC)
        self.lin_value = torch.nn.Linear(in_channels, HC)
        self.lin_edge = torch.nn.Linear(edge_dim, HC, bias=False) if edge_dim else None
        self.lin_skip = torch.nn.Linear(in_channels, HC if concat else out_channels) if root_weight else None
        self.use_kernel = use_kernel

    def forward(self, x: torch.Tensor, row_ptr: torch.Tensor, col: torch.Tensor,
                edge_attr: Optional[torch.Tensor] = None) -> torch.Tensor:
        n = x.shape[0]
        q, k, v = self.lin_query(x), self.lin_key(x), self.lin_value(x)
        w_e = self.lin_edge.weight[:, 0] if (self.lin_edge is not None and edge_attr is not None) else None
        ew = edge_attr.reshape(-1) if w_e is not None else None
        skip = self.lin_skip(x) if (self.lin_skip is not None and self.concat) else None
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if self.use_kernel and x.is_cuda and not grad:
            out = attn_aggregate(q.contiguous(), k.contiguous(), v.contiguous(), row_ptr, col.to(torch.int32),
                                 ew, w_e, skip, self.heads)
        else:
            out = attn_aggregate_ref(q, k, v, row_ptr, col, ew, w_e, skip, self.heads)
        if not self.concat:
            out = out.view(n, self.heads, self.out_channels).mean(1)
            if self.lin_skip is not None:
                out = out + self.lin_skip(x)
        return out
