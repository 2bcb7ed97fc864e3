"""Timeline of one segmented rollout launch at H (navigation, 24 agents x 8192
envs; diagnostic -DGSM_STAMPS build, run with GSM_LIB_PATH pointing at it):
per wave, s_memrealtime (100 MHz) at the marks of gsm_roll_seg_kernel —
0 entry, 1 state loaded, 2 step 0 physics, 3 step 0 sweep, 4 step K-1
published, 5 tail start, 6 step K-2 emitted, 7 step K-1 emitted, 8 final
state stored; 9 HW_ID | XCC_ID << 32 (where the wave ran); and s_memtime
cycles summed per phase over the steps (slots 10-14: the step's work, the
publish barrier, the CSR prefix of wave 0, the wait for it, staging +
emission). Prints, per mark, the percentiles over waves of the time
since the first wave's entry, for an eager env.step (a K = 1 launch) and for a
K-step graph replay (K = ROLL_K, default 20).

Usage: GSM_LIB_PATH=.../ablate/stamps.so python tools/stamps_h_timeline.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

B, N, T = 8192, 24, 100
K = int(os.environ.get("ROLL_K", 20))
dev = "cuda:0"
env = GpuBatchEnv(EnvConfig(scenario="navigation", n_agents=N, n_envs=B, seed=5, episode_length=T), dev)
st = torch.zeros(B, 16, dtype=torch.int64, device=dev)
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=dev)
env.reset(seed=5, sync_edges=False)
MARKS = ["entry", "loaded", "physics0", "sweep0", "published_last", "tail", "tail_emit1", "tail_emit2", "stored"]


def timeline():
    q = st.cpu().numpy().astype(np.int64)
    t0 = q[:, 0].min()
    out = {}
    for i, n in enumerate(MARKS):
        v = (q[:, i] - t0) / 100.0
        out[n] = {p: round(float(np.percentile(v, p)), 2) for p in (0, 50, 99, 100)}
    return out


res = {}
for _ in range(5):
    env.step(acts[0], sync_edges=False)
torch.cuda.synchronize()
st.zero_()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
env.step(acts[0], sync_edges=False)
e1.record()
torch.cuda.synchronize()
res["eager_step"] = {"events_us": e0.elapsed_time(e1) * 1e3, "marks_us": timeline()}
env.capture(acts, K, slot=0, kernels="roll")
for _ in range(3):
    env.replay(0)
# ROLL_START=s: the timed replay starts at step s of the episode (e.g. 90: it
# holds the episode boundary, every env auto-resetting in the same step)
start = int(os.environ.get("ROLL_START", 0))
env.reset(seed=5, sync_edges=False)
if start:
    env.capture(acts, start, slot=1, kernels="roll")
    env.replay(1)
torch.cuda.synchronize()
st.zero_()
e0.record()
env.replay(0)
e1.record()
torch.cuda.synchronize()
qq = st.cpu().numpy().astype(np.int64)
w0 = np.arange(B) % 4 == 0
PH = ["work", "publish_barrier", "prefix", "prefix_wait", "stage_emit"]
res[f"replay_K{K}_from{start}"] = {"events_us": e0.elapsed_time(e1) * 1e3, "marks_us": timeline(),
                       "wave0_cycles_per_step": {n: float(qq[w0, 10 + i].mean() / K) for i, n in enumerate(PH)},
                       "other_waves_cycles_per_step": {n: float(qq[~w0, 10 + i].mean() / K) for i, n in enumerate(PH)},
                       # slot 15: cycles in the re-layout block (auto-reset), summed over the launch
                       "relayout_cycles_per_launch": float(qq[:, 15].mean())}
hw = qq[:, 9]
if hw.any():
    # where each wave ran (slot 9: HW_ID | XCC_ID << 32) against when it
    # finished: the waves of one CU ranked by workgroup index (dispatch order)
    cu = ((hw >> 32) & 7) << 8 | ((hw >> 13) & 7) << 5 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15)
    simd = cu << 2 | ((hw >> 4) & 3)
    fin = (qq[:, 8] - qq[:, 0].min()) / 100.0
    wg = np.arange(B) // 4
    by_rank = {}
    for c in np.unique(cu):
        sel = np.nonzero(cu == c)[0]
        wgs = np.unique(wg[sel])
        for r, g in enumerate(wgs):
            by_rank.setdefault(r, []).append(float(fin[sel][wg[sel] == g].max()))
    res[f"replay_K{K}_from{start}"]["finish_us_by_rank_on_cu"] = {
        int(r): {"n": len(v), "mean": round(float(np.mean(v)), 2), "min": round(float(np.min(v)), 2),
                 "max": round(float(np.max(v)), 2)} for r, v in sorted(by_rank.items())}
    res[f"replay_K{K}_from{start}"]["cus"] = int(len(np.unique(cu)))
    res[f"replay_K{K}_from{start}"]["simds"] = int(len(np.unique(simd)))
    out = os.environ.get("STAMPS_NPZ")
    if out:
        np.savez_compressed(out, stamps=qq, hw=hw)
print(json.dumps(res, indent=1))
env.close()
