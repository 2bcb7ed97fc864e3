import sys, os, json
sys.path.insert(0, "gs-marl_amd")
import torch
from gsmarl_amd import EnvConfig, GpuBatchEnv
for seed, pre in ((3, 0), (1234, 0), (3, 250), (1234, 250)):
    env = GpuBatchEnv(EnvConfig(n_agents=24, n_envs=8192, seed=seed), "cuda:0")
    acts = torch.randint(0, 5, (100, 8192, 24), dtype=torch.int32, device="cuda:0")
    env.reset(seed=seed, sync_edges=False)
    if pre:
        env.capture(acts, pre, slot=1, kernels="both")
        env.replay(1)
    res = []
    for phase in range(4):
        env.capture(acts, 25, slot=0, kernels="lag", time_ends=True)
        env.replay(0); torch.cuda.synchronize()
        res.append(round(env.graph_kernel_ms(0)[0] * 1e3, 2))
    print(json.dumps(dict(seed=seed, pre=pre, lag_us_per_25step_block=res, edges=int(env.t["edge_ptr"][8192].item()) / 8192)))
    del env
