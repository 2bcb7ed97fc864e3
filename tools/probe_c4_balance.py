"""Ragged rollout time per step against the batch's mix: is a 100-step launch
bound by its most loaded SIMD? Times one 100-step rollout launch (events,
median of 3 after a warm launch) for uniform and mixed ragged batches, and
prints the model's per-SIMD load (env cost ~ a + b*N per family, envs placed
8 per SIMD in grid order) beside it.

Usage: python tools/probe_c4_balance.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

CASES = [("mixed", 24, 3, 8192), ("mixed", 24, 24, 8192), ("polygon", 24, None, 8192), ("line", 24, None, 8192),
         ("polygon", 12, None, 8192), ("line", 6, None, 8192), ("mixed", 24, 3, 4096), ("polygon", 24, None, 4096)]


def run(scn, N, nmin, B, T=100):
    kw = dict(scenario=scn, n_agents=N, n_envs=B, seed=5, episode_length=T)
    if nmin is not None:
        kw["n_agents_min"] = nmin
    env = GpuBatchEnv(EnvConfig(**kw), "cuda:0")
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device="cuda:0")
    env.reset(seed=5, sync_edges=False)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        s.record()
        env.replay(0)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / T)
    sh = env.t["env_shape"].cpu()
    n, sc = (sh & 0xFF).double(), (sh >> 8)
    cost = torch.where(sc == 0, 2000 + 700 * n, 4000 + 2900 * n)
    W = ((B + 3) // 4) * 4
    c = torch.zeros(W, dtype=torch.float64)
    c[:B] = cost
    per = W // 1024 if W >= 1024 else 1
    load = c[: (W // per) * per].reshape(-1, per).sum(1)
    res = dict(scenario=scn, N=N, n_min=nmin, B=B, us_per_step=round(statistics.median(ts), 2),
               gave_up=bool(env.roll_gave_up()), model_mean_load=round(float(load.mean()), 0),
               model_max_load_grid_order=round(float(load.max()), 0))
    env.close()
    return res


for case in CASES:
    print(json.dumps(run(*case)), flush=True)
