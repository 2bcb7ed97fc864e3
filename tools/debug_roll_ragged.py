"""Debug: ragged rollout (bound buffers) edge_ptr vs eager, the failing test's setup."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import torch
from gsmarl_amd import EnvConfig, GpuBatchEnv
DEV = "cuda:0"
B, N, T, EL = 300, 24, 11, 4
def fresh(env, seed):
    env.reset(seed=seed); env.t["lsa_v"].zero_(); env.t["lsa_col"].fill_(-1); env.t["lsa_stats"].zero_()
for depth in (8, 4, 8, 8, 6):
    os.environ["GSM_ROLL_DEPTH"] = str(depth)
    env = GpuBatchEnv(EnvConfig(scenario="mixed", n_agents=N, n_envs=B, seed=7, episode_length=EL), DEV)
    gen = torch.Generator(device=DEV); gen.manual_seed(B + T)
    acts = torch.randint(0, 5, (T - 2, B, N), dtype=torch.int32, device=DEV, generator=gen)
    fresh(env, 7)
    for t in range(T):
        env.step(acts[t % acts.shape[0]], sync_edges=False)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in env.t.items()}
    fresh(env, 7)
    env.capture(acts, T, slot=0, kernels="roll")
    env.t["edge_index"].fill_(-7)
    env.replay(0)
    torch.cuda.synchronize()
    d = env.t["edge_ptr"] - ref["edge_ptr"]
    w = d.nonzero().flatten().tolist()
    bad_keys = [k for k in ("pos", "vel", "edge_count", "row_mask", "assign", "node_feat") if not torch.equal(ref[k], env.t[k])]
    print("depth", depth, "gave_up", env.roll_gave_up(), "wrong ptr", len(w), w[:8], sorted(set(d[w].tolist()))[:5], "bad", bad_keys, flush=True)
    env.close()
