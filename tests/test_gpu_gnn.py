"""gsm_attn_aggregate (HIP, gsm_gnn.hip) vs the torch formulation
(gsmarl_amd.gnn.attn_aggregate_ref, fp32 and fp64) on random CSR graphs and on
the env's own graph at the headline size. Tolerance: 2e-5 absolute /
relative against fp64 (hardware exp in the online softmax)."""
import math

import numpy as np
import pytest
import torch

from gsmarl_amd import gnn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(n, rng, max_deg=6, empty=0.2):
    deg = rng.integers(0, max_deg + 1, size=n)
    deg[rng.random(n) < empty] = 0
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(deg, out=ptr[1:])
    col = rng.integers(0, n, size=int(ptr[-1])).astype(np.int32)
    return torch.from_numpy(ptr).to(DEV), torch.from_numpy(col).to(DEV)


@pytest.mark.parametrize("heads,C", [(1, 1), (1, 4), (2, 8), (3, 16), (4, 16), (2, 32), (1, 64)])
@pytest.mark.parametrize("edge,skip", [(True, True), (False, False)])
def test_kernel_matches_reference(heads, C, edge, skip):
    rng = np.random.default_rng(heads * 100 + C)
    n = 2000
    ptr, col = _graph(n, rng)
    HC = heads * C
    g = torch.Generator(device=DEV).manual_seed(3)
    q, k, v, sk = (torch.randn(n, HC, device=DEV, generator=g) for _ in range(4))
    ew = torch.rand(col.numel(), device=DEV, generator=g) if edge else None
    we = torch.randn(HC, device=DEV, generator=g) if edge else None
    s = sk if skip else None
    out = gnn.attn_aggregate(q, k, v, ptr, col, ew, we, s, heads)
    ref = gnn.attn_aggregate_ref(q.double(), k.double(), v.double(), ptr, col,
                                 ew.double() if edge else None, we.double() if edge else None,
                                 s.double() if skip else None, heads)
    err = (out.double() - ref).abs()
    assert torch.all(err <= 2e-5 * (1 + ref.abs())), float(err.max())
    empty = (ptr[1:] == ptr[:-1])
    base = s if skip else torch.zeros_like(q)
    assert torch.equal(out[empty], base[empty])          # no neighbours -> 0 (+ skip)


def test_env_graph_headline_size():
    """Message passing over the env's own COO output (symmetric, row-major =
    CSR over targets) at 24 agents x 8192 envs."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    env = GpuBatchEnv(EnvConfig(n_agents=24, n_envs=8192, seed=1), DEV)
    out = env.reset(seed=1)
    n = env.B * env.E
    ptr = gnn.env_csr(out["edge_index"], n)
    col = out["edge_index"][1].contiguous()
    conv = gnn.TransformerConv(7, 16, heads=3, concat=True).to(DEV)
    x = out["node_feat"].reshape(n, 7)
    with torch.no_grad():
        y = conv(x, ptr, col, out["edge_attr"].reshape(-1, 1))
        conv.use_kernel = False
        y_ref = conv(x, ptr, col, out["edge_attr"].reshape(-1, 1))
    assert y.shape == (n, 48)
    assert torch.allclose(y, y_ref, rtol=2e-5, atol=2e-5), float((y - y_ref).abs().max())
    env.close()


def test_rejects_unsupported_shapes():
    from gsmarl_amd._lib import GsmError
    q = torch.zeros(4, 48, device=DEV)
    ptr = torch.zeros(5, dtype=torch.int64, device=DEV)
    col = torch.zeros(0, dtype=torch.int32, device=DEV)
    with pytest.raises(GsmError):
        gnn.attn_aggregate(q, q, q, ptr, col, heads=1)        # C = 48: not a power of two
    with pytest.raises(GsmError):
        gnn.attn_aggregate(torch.zeros(4, 128, device=DEV), torch.zeros(4, 128, device=DEV),
                           torch.zeros(4, 128, device=DEV), ptr, col, heads=2)   # H*C > 64
