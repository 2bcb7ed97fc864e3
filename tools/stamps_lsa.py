"""Per-wave cycles and path iterations of the ragged kernel's assignment
(diagnostic -DGSM_STAMPS build: tools/build_variant.sh "stamps:-DGSM_STAMPS",
run with GSM_LIB_PATH pointing at it): one step of a polygon batch (ABL_N
agents, ABL_B envs), then the median s_memtime cycles spent in wave_lsa, the
median / max path iterations and the cycles per iteration."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gs-marl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402

N, B = int(os.environ.get("ABL_N", 24)), int(os.environ.get("ABL_B", 256))
scn = os.environ.get("ABL_SCN", "polygon")
env = GpuBatchEnv(EnvConfig(scenario=scn, n_agents=N, n_envs=B, seed=3), "cuda:0")
st = torch.zeros(max(B, 2 * env.sizes.n_blocks * 4), 16, dtype=torch.int64, device="cuda:0")
env.lib.gsm_debug_set_stamps(env._h, C.c_void_p(st.data_ptr()))
env.reset(seed=3, sync_edges=False)
for _ in range(int(os.environ.get("ABL_WARM", 5))):   # steps before the measured one (warm-start state)
    env.step(torch.randint(0, 5, (B, N), dtype=torch.int32, device="cuda:0"))
torch.cuda.synchronize()
st.zero_()
env.step(torch.randint(0, 5, (B, N), dtype=torch.int32, device="cuda:0"))
torch.cuda.synchronize()
s = st.cpu().numpy().astype(np.int64)[:B]
cyc, raw = s[:, 1] - s[:, 0], s[:, 2]
it, free = raw & 0xFFFF, (raw >> 16) & 0xFF
ok = cyc > 0
ph = np.diff(s[:, 4:8], axis=1)   # row loop, augments, certificate (s_memtime cycles)
pre = s[:, 4] - s[:, 0]           # cost matrix
print(json.dumps(dict(scenario=scn, N=N, B=B, envs=int(ok.sum()), lsa_cycles_median=float(np.median(cyc[ok])),
                      lsa_cycles_max=int(cyc[ok].max()),
                      iters_median=float(np.median(it[ok])), iters_max=int(it[ok].max()),
                      free_rows_median=float(np.median(free[ok])), free_rows_max=int(free[ok].max()),
                      warm_stats=env.lsa_warm_stats(),
                      phase_cycles_median=dict(cost=float(np.median(pre[ok])), rows=float(np.median(ph[ok, 0])),
                                               augment=float(np.median(ph[ok, 1])), certify=float(np.median(ph[ok, 2])),
                                               aug_loops=float(np.median(s[ok, 10])), aug_updates=float(np.median(s[ok, 11]))))))
