"""Per-wave phase accounting of the tile rollout kernel on the C3 batch
(navigation, 96 agents x 1024 envs; diagnostic -DGSM_STAMPS build, run with
GSM_LIB_PATH pointing at it). One 100-step launch after a warm one; per wave:
lifetime (s_memrealtime, 100 MHz) and s_memtime cycles summed per phase over
the steps (gsm_tile_kernels.hip gsm_roll_tile_kernel): physics, sweep (of which
the column pass), reward/cost exchange, node features + publish, look-back
(wave 0), emission, hand-over. Prints the mean per step of wave 0 and of the
other waves.

Usage: GSM_LIB_PATH=.../ablate/stamps.so python tools/stamps_c3_roll.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

B, N, T, WPB = 1024, 96, 100, 8
dev = "cuda:0"
env = GpuBatchEnv(EnvConfig(scenario="navigation", n_agents=N, n_envs=B, seed=5, episode_length=T), dev)
st = torch.zeros(B * WPB, 16, dtype=torch.int64, device=dev)
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=dev)
env.reset(seed=5, sync_edges=False)
env.capture(acts, T, slot=0, kernels="roll")
env.replay(0)
torch.cuda.synchronize()
st.zero_()
s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s0.record()
env.replay(0)
s1.record()
torch.cuda.synchronize()
assert not env.roll_gave_up()
q = st.cpu().numpy().astype(np.int64)
names = ["physics", "sweep_columns", "sweep", "reward_exchange", "nodefeat_publish", "lookback", "emit", "handover"]
t0 = q[:, 8].min()
start, end = (q[:, 8] - t0) / 100.0, (q[:, 9] - t0) / 100.0
w0 = np.arange(B * WPB) % WPB == 0
out = {"launch_ms_events": s0.elapsed_time(s1), "span_us": float(end.max()), "start_max_us": float(start.max()),
       "lifetime_us_p50": float(np.median(end - start)),
       "wave0_cycles_per_step": {n: float(q[w0, i].mean() / T) for i, n in enumerate(names)},
       "other_waves_cycles_per_step": {n: float(q[~w0, i].mean() / T) for i, n in enumerate(names)},
       "lifetime_cycles_per_step_p50_est": float(np.median(q[:, :8].sum(1) - q[:, 1]) / T)}
print(json.dumps(out, indent=1))
env.close()
