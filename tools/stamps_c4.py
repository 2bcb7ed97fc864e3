"""Per-wave timeline of the ragged step kernel on the mixed C4 batch
(diagnostic -DGSM_STAMPS build; run with GSM_LIB_PATH pointing at it): one
step after ABL_WARM warm steps; per (scenario, N) group the median wave
lifetime and assignment cycles, and when the last waves start / end."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gs-marl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

B = int(os.environ.get("ABL_B", 8192))
env = GpuBatchEnv(EnvConfig(scenario="mixed", n_agents=24, n_envs=B, seed=3), "cuda:0")
st = torch.zeros(max(B, 2 * env.sizes.n_blocks * 4), 16, dtype=torch.int64, device="cuda:0")
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
env.reset(seed=3, sync_edges=False)
for _ in range(int(os.environ.get("ABL_WARM", 5))):
    env.step(torch.randint(0, 5, (B, 24), dtype=torch.int32, device="cuda:0"))
torch.cuda.synchronize()
res = []
for rep in range(int(os.environ.get("ABL_REPS", 1))):
    st.zero_()
    env.step(torch.randint(0, 5, (B, 24), dtype=torch.int32, device="cuda:0"))
    torch.cuda.synchronize()
    q = st.cpu().numpy().astype(np.int64)[:B]
    code = (q[:, 2] >> 24) & 0xFF
    sc = q[:, 3] >> 8
    res.append([int(((sc > 0) & (code == c)).sum()) for c in range(5)])
print("cert codes per step (none, ok, infeasible, cycle):", res)
st.zero_()
env.step(torch.randint(0, 5, (B, 24), dtype=torch.int32, device="cuda:0"))
torch.cuda.synchronize()
s = st.cpu().numpy().astype(np.int64)[:B]
t0 = s[:, 8].min()
start, end = (s[:, 8] - t0) / 100.0, (s[:, 9] - t0) / 100.0   # us (100 MHz realtime)
lsa = s[:, 1] - s[:, 0]
N, scn = s[:, 3] & 0xFF, s[:, 3] >> 8
out = {"span_us": float(end.max()), "start_p50": float(np.median(start)), "start_max": float(start.max()),
       "end_p50": float(np.median(end)), "groups": {}}
for sc in (0, 1, 2):
    for n in (3, 8, 12, 16, 20, 24):
        m = (scn == sc) & (N == n)
        if m.any():
            out["groups"][f"scn{sc}_N{n}"] = dict(
                count=int(m.sum()), life_us_p50=float(np.median(end[m] - start[m])),
                life_us_max=float((end[m] - start[m]).max()), start_us_max=float(start[m].max()),
                end_us_max=float(end[m].max()), lsa_cyc_p50=float(np.median(lsa[m])) if sc else 0.0,
                iters_p50=float(np.median(s[m, 2] & 0xFFFF)), free_p50=float(np.median((s[m, 2] >> 16) & 0xFF)))
code = (s[:, 2] >> 24) & 0xFF
out["cert_codes"] = {str(c): int((code[scn > 0] == c).sum()) for c in range(5)}
out["uncertified"] = [dict(N=int(N[i]), scn=int(scn[i]), code=int(code[i]), start=float(start[i]), end=float(end[i]),
                           iters=int(s[i, 2] & 0xFFFF)) for i in np.where((scn > 0) & (code != 1))[0][:20]]
bad = np.where((scn > 0) & (code != 1))[0]
if len(bad):   # state of the tied envs (post-step positions) for offline analysis
    st_ = env.get_state()
    out["tied_states"] = [dict(b=int(i), N=int(N[i]), scn=int(scn[i]),
                               pos=st_["pos"][i].cpu().numpy().view(np.uint32).tolist()) for i in bad[:4]]
late = np.argsort(end)[-8:]
out["last_enders"] = [dict(N=int(N[i]), scn=int(scn[i]), start=float(start[i]), end=float(end[i])) for i in late]
print(json.dumps(out, indent=1))
