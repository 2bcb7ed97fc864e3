import sys; sys.path.insert(0, "gs-marl_amd")
import torch
from gsmarl_amd import EnvConfig, GpuBatchEnv
env = GpuBatchEnv(EnvConfig(n_agents=3, n_envs=8), "cuda:0")
env.reset(seed=0)
a = torch.zeros(4, 8, 3, dtype=torch.int32, device="cuda:0")
for n in (1, 2, 3):
    try:
        env.capture(a, n, timing=True, slot=0); env.replay(0); torch.cuda.synchronize()
        print(n, "ok", env.graph_kernel_ms(0))
    except Exception as e:
        print(n, "FAIL", e)
