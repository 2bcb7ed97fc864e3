"""Debug: rollout vs eager for small K at two 64-wave groups (slot and bound modes)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]
import torch
from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
DEV = "cuda:0"
for N, B, T, mode in [(3, 100, 1, "slots"), (3, 100, 1, "bound"), (3, 100, 2, "slots"), (24, 100, 1, "slots"), (24, 100, 1, "bound"), (3, 100, 3, "slots")]:
    for rep in range(2):
        env = GpuBatchEnv(EnvConfig(n_agents=N, n_envs=B, seed=2, episode_length=6), DEV)
        ref = GpuBatchEnv(EnvConfig(n_agents=N, n_envs=B, seed=2, episode_length=6), DEV)
        acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
        if mode == "slots":
            gb = GraphRolloutBuffer(env, episode_length=T); eb = GraphRolloutBuffer(ref, episode_length=T)
            gb.reset(seed=2); gb.capture(acts); gb.replay()
            eb.reset(seed=2)
            for t in range(T): eb.insert(acts[t])
            torch.cuda.synchronize()
            g, e = gb.edge_ptr[T], eb.edge_ptr[T]
        else:
            env.reset(seed=2); env.capture(acts, T, slot=0, kernels="roll"); env.replay(0)
            ref.reset(seed=2)
            for t in range(T): ref.step(acts[t], sync_edges=False)
            torch.cuda.synchronize()
            g, e = env.t["edge_ptr"], ref.t["edge_ptr"]
        bad = (g != e).nonzero().flatten().tolist()
        print(N, B, T, mode, rep, "gave_up", env.roll_gave_up(), "wrong", bad[:20], "diff", (e - g)[bad[:5]].tolist() if bad else [], flush=True)
        env.close(); ref.close()
