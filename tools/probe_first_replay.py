"""Probe: wall-clock of successive replays of ONE captured rollout graph
(20 steps at the headline shape), each bracketed by synchronize — does the
first replay of a freshly captured graph pay a one-time cost that the
driver's 20-step bench line (one replay in its timed region) absorbs?

Usage: python tools/probe_first_replay.py [steps] [replays]
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gs-marl_amd"))

import torch  # noqa: E402
from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(seed=1234, n_agents=24, n_envs=8192)
    env = GpuBatchEnv(cfg, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)
    actions = torch.randint(0, 5, (cfg.episode_length, 8192, 24), dtype=torch.int32, device=dev, generator=gen)
    env.reset(seed=cfg.seed, sync_edges=False)
    env.capture(actions, 5, timing=False, slot=2, kernels="roll")
    env.replay(2)             # the kernels' first use (code objects loaded)
    torch.cuda.synchronize(dev)
    env.capture(actions, K, timing=False, slot=0, kernels="roll")
    torch.cuda.synchronize(dev)
    out = []
    for _ in range(R):
        t0 = time.perf_counter()
        env.replay(0)
        torch.cuda.synchronize(dev)
        out.append(round((time.perf_counter() - t0) * 1e6, 1))
    idle = []
    for _ in range(4):   # synchronize alone: the host's round trip
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        idle.append(round((time.perf_counter() - t0) * 1e6, 1))
    print(json.dumps({"steps": K, "replay_us": out, "sync_only_us": idle,
                      "gave_up": bool(env.roll_gave_up())}))
    env.close()


if __name__ == "__main__":
    main()
