"""Per-wave phase accounting of the packed small-env rollout kernel on the C2
batch (navigation, 3 agents x 4096 envs, four envs per wave; diagnostic
-DGSM_STAMPS build, run with GSM_LIB_PATH pointing at it). One 100-step launch
after a warm one; per wave, s_memtime cycles summed per phase over the steps
(gsm_seg_kernels.hip gsm_roll_pack_kernel): the step's work, the hand-off
publishes, the settle of the offset granules, the emission; and the lifetime
(s_memrealtime, 100 MHz).

Usage: GSM_LIB_PATH=.../ablate/stamps.so python tools/stamps_c2_roll.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

B, N, T = 4096, 3, 100
dev = "cuda:0"
env = GpuBatchEnv(EnvConfig(scenario="navigation", n_agents=N, n_envs=B, seed=5, episode_length=T), dev)
W = B // 4
st = torch.zeros(W, 16, dtype=torch.int64, device=dev)
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
if q[:, 10].any():   # gsm_roll_pack2_kernel: stepping and emitting waves
    t0 = min(q[:, 8].min(), q[:, 10].min())
    names = {0: "step_work", 1: "publish", 2: "ring_wait", 3: "emitter_wait_step", 5: "emitter_offset_settle",
             4: "emitter_emit"}
    out = {"launch_ms_events": s0.elapsed_time(s1),
           "stepper_span_us_max": float(((q[:, 9] - t0) / 100.0).max()),
           "emitter_span_us_max": float(((q[:, 11] - t0) / 100.0).max()),
           "stepper_end_us_p50": float(np.median((q[:, 9] - t0) / 100.0)),
           "emitter_end_us_p50": float(np.median((q[:, 11] - t0) / 100.0)),
           "cycles_per_step_mean": {n: float(q[:, i].mean() / T) for i, n in names.items()},
           "cycles_per_step_p99": {n: float(np.percentile(q[:, i] / T, 99)) for i, n in names.items()}}
    print(json.dumps(out, indent=1))
    env.close()
    sys.exit(0)
names = ["work", "publish", "unused", "offset_settle", "emit"]
t0 = q[:, 8].min()
start, end = (q[:, 8] - t0) / 100.0, (q[:, 9] - t0) / 100.0
w0 = np.arange(W) % 4 == 0
out = {"launch_ms_events": s0.elapsed_time(s1), "span_us": float(end.max()), "start_max_us": float(start.max()),
       "loop_us_p50": float(np.median(end - start)),
       "wave0_cycles_per_step": {n: float(q[w0, i].mean() / T) for i, n in enumerate(names)},
       "other_waves_cycles_per_step": {n: float(q[~w0, i].mean() / T) for i, n in enumerate(names)}}
print(json.dumps(out, indent=1))
env.close()
