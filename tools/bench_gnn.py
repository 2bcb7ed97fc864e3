"""Measure gsm_attn_aggregate (the GNN message-passing kernel) on the env's
own graph at the headline size (24 agents x 8192 envs: 589,824 nodes), and
the torch formulation of the same op for comparison. One JSON line.

Algorithmic bytes per launch: q, skip and out rows once per node (3 x 4HC),
k and v rows once per node (each row is gathered by its ~2.5 neighbours, which
sit in the same env, so one HBM read), row_ptr (8) per node, col + edge
weight (8) per edge."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gs-marl_amd"))
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv, gnn  # noqa: E402

DEV = "cuda:0"
heads, C = int(os.environ.get("GNN_HEADS", 3)), int(os.environ.get("GNN_C", 16))
B = int(os.environ.get("GNN_B", 8192))
env = GpuBatchEnv(EnvConfig(n_agents=24, n_envs=B, seed=1), DEV)
out = env.reset(seed=1)
n = env.B * env.E
ptr = gnn.env_csr(out["edge_index"], n)
col = out["edge_index"][1].contiguous()
ew = out["edge_attr"].contiguous()
nE = col.numel()
HC = heads * C
g = torch.Generator(device=DEV).manual_seed(0)
q, k, v, sk = (torch.randn(n, HC, device=DEV, generator=g) for _ in range(4))
we = torch.randn(HC, device=DEV, generator=g)


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


kern_ms = timed(lambda: gnn.attn_aggregate(q, k, v, ptr, col, ew, we, sk, heads), 100)
ref_ms = timed(lambda: gnn.attn_aggregate_ref(q, k, v, ptr, col, ew, we, sk, heads), 10)
bytes_ = n * (3 * 4 * HC + 2 * 4 * HC + 8) + nE * 8
ach = bytes_ / (kern_ms * 1e-3) / 1e9
print(json.dumps({
    "op": "gsm_attn_aggregate (TransformerConv edge softmax + aggregation)",
    "graph": f"env graph, 24 agents x {B} envs: {n} nodes, {nE} edges",
    "heads": heads, "channels": C, "kernel_us": round(kern_ms * 1e3, 2),
    "torch_formulation_us": round(ref_ms * 1e3, 1), "speedup_vs_torch": round(ref_ms / kern_ms, 1),
    "algorithmic_bytes": int(bytes_), "achieved_GBs": round(ach, 1), "frac_of_8TBs": round(ach / 8000, 4),
    "timing": "torch.cuda events around 100 launches on the current stream (the kernel's stream)",
}))
env.close()
