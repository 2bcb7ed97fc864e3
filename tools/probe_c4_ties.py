"""C4 (mixed, 24 x 8192): do the envs whose assignment fell back to the cold
solve (a tie) fall back again on the next step? Per env and step, cold =
assignments solved - certified warm starts (the lsa_stats counters).
Usage: python tools/probe_c4_ties.py [--T 60]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]

import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=60)
    a = ap.parse_args()
    env = GpuBatchEnv(EnvConfig(scenario="mixed", n_agents=24, n_agents_min=3, n_envs=8192, seed=1234), "cuda:0")
    env.reset(seed=1234, sync_edges=False)
    prev = env.t["lsa_stats"].clone()
    colds = []
    for t in range(a.T):
        env.step(torch.randint(0, 5, (8192, 24), dtype=torch.int32, device="cuda:0"), sync_edges=False)
        cur = env.t["lsa_stats"].clone()
        d = cur - prev
        colds.append((d[:, 1] - d[:, 0]) > 0)
        prev = cur
    torch.cuda.synchronize()
    c = torch.stack(colds).cpu()
    again = (c[:-1] & c[1:]).sum().item()
    n = c[:-1].sum().item()
    per_env = c.sum(0)
    out = {"steps": a.T, "cold_per_step": round(c.sum().item() / a.T, 2), "cold_then_cold": again, "cold": n,
           "p_again": round(again / max(n, 1), 3), "envs_ever_cold": int((per_env > 0).sum()),
           "max_cold_steps_one_env": int(per_env.max())}
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
