"""CPU checks of the GNN aggregation's torch formulation (gsmarl_amd.gnn):
against a per-node Python loop of the TransformerConv equations, empty rows,
gradients, and the env-graph CSR helper."""
import math

import numpy as np
import torch

from gsmarl_amd import gnn


def _graph(n, rng, max_deg=5, empty=0.2):
    deg = rng.integers(0, max_deg + 1, size=n)
    deg[rng.random(n) < empty] = 0
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(deg, out=ptr[1:])
    col = rng.integers(0, n, size=int(ptr[-1])).astype(np.int32)
    return torch.from_numpy(ptr), torch.from_numpy(col)


def _loop(q, k, v, ptr, col, ew, we, skip, heads, scale):
    n, HC = q.shape
    Cc = HC // heads
    out = torch.zeros_like(q)
    for i in range(n):
        for h in range(heads):
            sl = slice(h * Cc, (h + 1) * Cc)
            s, vals = [], []
            for t in range(int(ptr[i]), int(ptr[i + 1])):
                j = int(col[t])
                e = ew[t] * we[sl] if ew is not None else 0.0
                s.append(float((q[i, sl] * (k[j, sl] + e)).sum()) * scale)
                vals.append(v[j, sl] + e)
            if s:
                m = max(s)
                w = [math.exp(x - m) for x in s]
                out[i, sl] = sum(wi * vi for wi, vi in zip(w, vals)) / sum(w)
    return out + (skip if skip is not None else 0)


def test_ref_matches_loop():
    rng = np.random.default_rng(0)
    for heads, Cc in ((1, 4), (3, 2), (2, 8)):
        n = 23
        ptr, col = _graph(n, rng)
        HC = heads * Cc
        q, k, v, skip = (torch.randn(n, HC, dtype=torch.float64) for _ in range(4))
        ew = torch.rand(col.numel(), dtype=torch.float64)
        we = torch.randn(HC, dtype=torch.float64)
        sc = 1 / math.sqrt(Cc)
        ref = gnn.attn_aggregate_ref(q, k, v, ptr, col, ew, we, skip, heads)
        assert torch.allclose(ref, _loop(q, k, v, ptr, col, ew, we, skip, heads, sc), atol=1e-12)
        ref0 = gnn.attn_aggregate_ref(q, k, v, ptr, col, heads=heads)
        assert torch.allclose(ref0, _loop(q, k, v, ptr, col, None, None, None, heads, sc), atol=1e-12)


def test_ref_gradients_and_module():
    rng = np.random.default_rng(1)
    ptr, col = _graph(30, rng)
    conv = gnn.TransformerConv(7, 16, heads=3, concat=False)
    x = torch.randn(30, 7, requires_grad=True)
    out = conv(x, ptr, col, torch.rand(col.numel(), 1))
    assert out.shape == (30, 16)
    out.sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    assert conv.lin_edge.weight.grad is not None


def test_env_csr():
    ei = torch.tensor([[0, 0, 2, 5, 5, 5], [1, 2, 0, 1, 2, 3]])
    assert gnn.env_csr(ei, 7).tolist() == [0, 2, 2, 3, 3, 3, 6, 6]
