"""Time the step/emit kernels of several libgsm builds (variants compiled with
-D flags by tools/ablate.sh) on the headline config, one process per build.
Prints mean kernel ms from the timed HIP graph (event nodes)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gs-marl_amd"))
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

N, B = int(os.environ.get("ABL_N", 24)), int(os.environ.get("ABL_B", 8192))
env = GpuBatchEnv(EnvConfig(n_agents=N, n_envs=B, seed=3), "cuda:0")
acts = torch.randint(0, 5, (100, B, N), dtype=torch.int32, device="cuda:0")
env.reset(seed=3, sync_edges=False)
env.capture(acts, 100, timing=True, slot=0)
res = []
for rep in range(5):
    env.replay(0)
    torch.cuda.synchronize()
    res.append(env.graph_kernel_ms(0))
s = sorted(r[0] for r in res)[2]
e = sorted(r[1] for r in res)[2]
print(json.dumps({"lib": os.environ.get("GSM_LIB_PATH", "default"), "step_ms": s, "emit_ms": e}))
