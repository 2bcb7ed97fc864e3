"""Fused rollout vs lagged chain at a given batch: whole-graph time per step
(HIP events around the graph) and the rollout kernel alone (events around its
launch). Usage: python tools/probe_roll.py [--B 8192] [--N 24] [--T 100]."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]

import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402


def timed(env, slot, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    env.replay(slot)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        env.replay(slot)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--N", type=int, default=24)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sweep", action="store_true", help="whole-graph time vs graph length (fixed cost)")
    ap.add_argument("--buffer", action="store_true",
                    help="also an episode into a GraphRolloutBuffer (per-step slots) via capture_into")
    a = ap.parse_args()
    env = GpuBatchEnv(EnvConfig(n_agents=a.N, n_envs=a.B, seed=1234), "cuda:0")
    acts = torch.randint(0, 5, (100, a.B, a.N), dtype=torch.int32, device="cuda:0")
    env.reset(seed=1234, sync_edges=False)
    out = {"B": a.B, "N": a.N, "T": a.T}
    if a.sweep:
        for kern in ("both", "roll"):
            for T in (1, 2, 5, 20, 100):
                env.capture(acts, T, slot=0, kernels=kern)
                out[f"{kern}_T{T}_graph_us"] = round(timed(env, 0, a.reps) * 1e3, 2)
    for kern in ("both", "roll"):
        env.capture(acts, a.T, slot=0, kernels=kern)
        ms = timed(env, 0, a.reps)
        out[f"{kern}_graph_us_per_step"] = round(ms * 1e3 / a.T, 3)
    env.capture(acts, a.T, slot=1, kernels="roll", time_ends=True)
    env.replay(1)
    torch.cuda.synchronize()
    out["roll_kernel_us_per_step"] = round(env.graph_kernel_ms(1)[0] * 1e3, 3)
    if a.buffer:   # every step's outputs into its own slot (distinct addresses)
        from gsmarl_amd import GraphRolloutBuffer
        buf = GraphRolloutBuffer(env, episode_length=a.T)
        buf.reset(seed=1234)
        buf.capture(acts[: a.T], slot=2)
        out["buffer_fused"] = env.graph_is_rollout(2)
        out["buffer_graph_us_per_step"] = round(timed(env, 2, a.reps) * 1e3 / a.T, 3)
        out["buffer_overflowed"] = bool(buf.overflowed())
    out["gave_up"] = env.roll_gave_up()
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
