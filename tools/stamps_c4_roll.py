"""Per-wave accounting of the ragged rollout kernel on the C4 batch (mixed,
N in {3..24} x 8192; diagnostic -DGSM_STAMPS build, run with GSM_LIB_PATH
pointing at it). One 100-step launch after a warm one; per wave: lifetime
(s_memrealtime, 100 MHz), s_memtime cycles summed per phase over the steps
(physics, group-sum publish, sweep + slab publish, assignment, pack), cold
solves (lsa_stats), and where it ran (HW_ID / XCC_ID). Prints the phase
split, the per-SIMD load spread and the last waves to finish.

Usage: GSM_LIB_PATH=.../ablate/stamps.so python tools/stamps_c4_roll.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

B, N, T = int(os.environ.get("ABL_B", 8192)), 24, 100
dev = "cuda:0"
env = GpuBatchEnv(EnvConfig(scenario="mixed", n_agents=N, n_envs=B, n_agents_min=3, seed=5, episode_length=T), dev)
W = ((B + 3) // 4) * 4
st = torch.zeros(W, 16, dtype=torch.int64, device=dev)
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=dev)
env.reset(seed=5, sync_edges=False)
env.capture(acts, T, slot=0, kernels="roll")
env.replay(0)
torch.cuda.synchronize()
shape = env.t["env_shape"].cpu().numpy()[:B]
stats0 = env.t["lsa_stats"].cpu().numpy().astype(np.int64)
st.zero_()
s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s0.record()
env.replay(0)
s1.record()
torch.cuda.synchronize()
assert not env.roll_gave_up()
stats1 = env.t["lsa_stats"].cpu().numpy().astype(np.int64)
q = st.cpu().numpy().astype(np.int64)[:B]
cold = (stats1[:, 1] - stats0[:, 1]) - (stats1[:, 0] - stats0[:, 0])
t0 = q[:, 0].min()
start, loop_end, end = (q[:, 0] - t0) / 100.0, (q[:, 1] - t0) / 100.0, (q[:, 2] - t0) / 100.0
ph = {"physics": q[:, 3], "grp_publish": q[:, 5], "sweep_publish": q[:, 4], "assign": q[:, 6], "pack": q[:, 7]}
hw, xcc = q[:, 8], q[:, 9]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
simd_key = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
scn, n = shape >> 8, shape & 0xFF
tot = sum(ph.values())
qq = st.cpu().numpy().astype(np.int64)
dec = qq[:W, 12]
out0 = {"placement_decisions": {str(int(k)): int(v) for k, v in zip(*np.unique(dec, return_counts=True))},
        "placement_wait_us_max": float(qq[:W, 13].max() / 100.0), "placement_wait_us_p50": float(np.median(qq[:W, 13]) / 100.0)}
out = {**out0, "launch_ms_events": s0.elapsed_time(s1), "span_us": float(end.max()), "start_max_us": float(start.max()),
       "end_p50_us": float(np.median(end)), "end_p99_us": float(np.percentile(end, 99)),
       "loop_end_max_us": float(loop_end.max()),
       "phase_cycles_mean_per_step": {k: float(v.mean() / T) for k, v in ph.items()},
       "phase_cycles_p99_per_step": {k: float(np.percentile(v, 99) / T) for k, v in ph.items()},
       "cold_solves": int(cold.sum())}
# per-SIMD: the sum of its waves' non-wait cycles (physics + sweep + assign)
work = ph["physics"] + ph["sweep_publish"] + ph["assign"]
keys, inv = np.unique(simd_key, return_inverse=True)
per_simd = np.bincount(inv, weights=work.astype(np.float64))
waves_per = np.bincount(inv)
out["simds"] = int(len(keys))
out["waves_per_simd"] = {str(int(k)): int(v) for k, v in zip(*np.unique(waves_per, return_counts=True))}
out["simd_work_cycles_per_step"] = dict(mean=float(per_simd.mean() / T), max=float(per_simd.max() / T),
                                         p50=float(np.median(per_simd) / T))
groups = {}
for sc in (0, 1, 2):
    for lo, hi in ((3, 8), (9, 16), (17, 24)):
        m = (scn == sc) & (n >= lo) & (n <= hi)
        if m.any():
            groups[f"scn{sc}_N{lo}-{hi}"] = dict(count=int(m.sum()), end_p50=float(np.median(end[m])),
                                                  end_max=float(end[m].max()),
                                                  work_per_step=float(np.median(work[m]) / T),
                                                  assign_per_step=float(np.median(ph["assign"][m]) / T),
                                                  wait_per_step=float(np.median(ph["grp_publish"][m] + ph["pack"][m]) / T))
out["groups"] = groups
late = np.argsort(end)[-10:]
out["last_enders"] = [dict(w=int(i), N=int(n[i]), scn=int(scn[i]), cold=int(cold[i]), end=float(end[i]),
                           work_per_step=float(work[i] / T), wait_per_step=float((ph["grp_publish"][i] + ph["pack"][i]) / T),
                           simd_work_per_step=float(per_simd[inv[i]] / T)) for i in late]
out["simd_work_max_over_mean"] = float(per_simd.max() / per_simd.mean())
if os.environ.get("STAMPS_NPZ"):   # per-env arrays for offline fits of the placement cost model
    np.savez(os.environ["STAMPS_NPZ"], scn=scn, n=n, work=work, assign=ph["assign"], physics=ph["physics"],
             sweep=ph["sweep_publish"], cold=cold, simd_key=simd_key, end=end)
print(json.dumps(out, indent=1))
env.close()
