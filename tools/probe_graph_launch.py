import sys, time, os
sys.path.insert(0, "gs-marl_amd")
import torch
from gsmarl_amd import EnvConfig, GpuBatchEnv
env = GpuBatchEnv(EnvConfig(n_agents=24, n_envs=int(os.environ.get("B", "64")), seed=3), "cuda:0")
B = env.cfg.n_envs
acts = torch.randint(0, 5, (100, B, 24), dtype=torch.int32, device="cuda:0")
env.reset(seed=3, sync_edges=False)
for n in (1, 2, 5, 10, 20, 50, 100):
    env.capture(acts, n, timing=False, slot=0)
    env.replay(0); torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter(); env.replay(0); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"B={B} steps={n}: median {ts[10]*1e6:.1f} us, per step {ts[10]*1e6/n:.2f} us")
