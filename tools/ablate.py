"""Time the step/emit kernels of several libgsm builds (variants compiled with
-D flags by tools/ablate.sh), one process per build: mean kernel ms over 100
back-to-back launches of each kernel (HIP events at the graph ends), plus the
whole-step ms of a 100-step graph. ABL_N / ABL_B / ABL_SCN pick the config."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gs-marl_amd"))
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

N, B = int(os.environ.get("ABL_N", 24)), int(os.environ.get("ABL_B", 8192))
scn = os.environ.get("ABL_SCN", "navigation")
env = GpuBatchEnv(EnvConfig(scenario=scn, n_agents=N, n_envs=B, seed=3), "cuda:0")
acts = torch.randint(0, 5, (100, B, N), dtype=torch.int32, device="cuda:0")
env.reset(seed=3, sync_edges=False)


def med(kernels, idx):
    env.capture(acts if kernels != "emit" else None, 100, slot=0, kernels=kernels, time_ends=True)
    res = []
    for _ in range(5):
        env.replay(0)
        torch.cuda.synchronize()
        res.append(env.graph_kernel_ms(0)[idx])
    return sorted(res)[2]


s = med("step", 0)
e = med("emit", 1)
out = {"lib": os.environ.get("GSM_LIB_PATH", "default"), "N": N, "B": B, "scenario": scn,
       "step_ms": s, "emit_ms": e, "step_total_ms_unfused": med("unfused", 2) / 100}
if not env.cfg.ragged and env.sizes.n_colliders <= 64:   # segmented: lagged emission
    out["lag_step_ms"] = med("lag", 0)
out["step_total_ms"] = med("both", 2) / 100
print(json.dumps(out))
