"""Why does the h line's timed region cost ~0.9 us per step more than the
roofline's settled launches (7.7 vs 6.8 us)? Two 100-step rollout graphs of
the same env in two slots (as bench.py's slot 0 and slot 3), timed
alternately: HIP events around three back-to-back replays, events around a
single replay, and the wall time of three replays between two synchronizes
(the timed region's form). Prints one JSON line per measurement round.

Usage: python tools/probe_slots.py [--rounds 5] [--offset 50]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]

import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--offset", type=int, default=0, help="eager steps before the captures: where the "
                    "synchronised episode boundary falls in each 100-step launch")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, N, EL = 8192, 24, 100
    env = GpuBatchEnv(EnvConfig(n_agents=N, n_envs=B, seed=1234, episode_length=EL), dev)
    env.reset(sync_edges=False)
    g = torch.Generator(device=dev).manual_seed(7)
    acts = torch.randint(0, 5, (EL, B, N), dtype=torch.int32, device=dev, generator=g)
    for t in range(a.offset):
        env.step(acts[t % EL], sync_edges=False)
    for slot in (0, 3):
        env.capture(acts, EL, slot=slot, kernels="roll")
    t_s = time.perf_counter()
    while time.perf_counter() - t_s < 2.0:   # settle, as bench.py does
        env.replay(0)
        torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def ev3(slot):
        e[0].record()
        for _ in range(3):
            env.replay(slot)
        e[1].record()
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) * 1e3 / 3

    def ev1(slot):
        env.replay(slot)
        env.replay(slot)
        e[0].record()
        env.replay(slot)
        e[1].record()
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) * 1e3

    def wall3(slot):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            env.replay(slot)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / 3

    for r in range(a.rounds):
        out = {"round": r, "offset": a.offset}
        for slot in (0, 3):
            out[f"s{slot}_ev3"] = round(ev3(slot), 1)
            out[f"s{slot}_ev1"] = round(ev1(slot), 1)
            out[f"s{slot}_wall3"] = round(wall3(slot), 1)
        print(json.dumps(out), flush=True)
    assert not env.roll_gave_up()
    env.close()


if __name__ == "__main__":
    main()
