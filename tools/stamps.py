"""Per-phase wave timelines from a -DGSM_STAMPS build (tools/build_variant.sh
"stamps:-DGSM_STAMPS"). Runs one timed 100-step graph on the headline config
and summarises the last step's stamps (diagnostic only; stamps perturb timing).
Step-kernel phases (gsm_seg_kernels.hip): 0 entry, 1 inputs staged, 2 lagged
emission done, 3 physics, 4 sweep, 5 reward/cost/auto-reset, 6 node features
and state stores, 7 counters."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gs-marl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

N, B = int(os.environ.get("ABL_N", 24)), int(os.environ.get("ABL_B", 8192))
env = GpuBatchEnv(EnvConfig(n_agents=N, n_envs=B, seed=3), "cuda:0")
nb = env.sizes.n_blocks
st = torch.zeros(2 * nb * 4, 16, dtype=torch.int64, device="cuda:0")
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
acts = torch.randint(0, 5, (100, B, N), dtype=torch.int32, device="cuda:0")
env.reset(seed=3, sync_edges=False)
env.capture(acts, int(os.environ.get("ABL_T", 99)), timing=False, slot=0)
env.replay(0)
torch.cuda.synchronize()
s = st.cpu().numpy().astype(np.int64)
out = {}
for name, rows, phases in (("step", s[: nb * 4], 8), ("emit", s[nb * 4:], 5)):
    live = rows[rows[:, 0] != 0]
    d = np.diff(live[:, :phases], axis=1)
    rt0, rt1 = live[:, 8], live[:, 9]
    out[name] = dict(
        waves=int(len(live)),
        phase_cycles_median=[int(x) for x in np.median(d, axis=0)],
        phase_cycles_mean=[int(x) for x in d.mean(axis=0)],
        wave_total_cycles_median=int(np.median(live[:, phases - 1] - live[:, 0])),
        start_spread_us=float((rt0.max() - rt0.min()) / 100.0),
        span_us=float((rt1.max() - rt0.min()) / 100.0),
        wave_lifetime_us_median=float(np.median(rt1 - rt0) / 100.0),
        phase_cycles_p90=[int(x) for x in np.percentile(d, 90, axis=0)],
        start_us_pct=[float(x) for x in np.percentile((rt0 - rt0.min()) / 100.0, [10, 50, 90, 100])],
        end_us_pct=[float(x) for x in np.percentile((rt1 - rt0.min()) / 100.0, [10, 50, 90, 100])],
    )
print(json.dumps(out, indent=1))
