"""Eager env.step at H (24 agents x 8192 envs): host issue time per step (the
loop without a sync) against device time per step (the loop with a sync at
both ends), and the same for bare gsm_step calls through the C-ABI (no
Python wrapper). Prints one JSON line. Run as
    python tools/probe_eager.py [--steps 2000]
with GSM_EAGER_ONE_LAUNCH=1 for the one-launch form."""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gs-marl_amd"))

import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--agents", type=int, default=24)
    ap.add_argument("--envs", type=int, default=8192)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = EnvConfig(n_agents=a.agents, n_envs=a.envs, seed=1234)
    env = GpuBatchEnv(cfg, dev)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(5)
    acts = torch.randint(0, 5, (100, a.envs, a.agents), dtype=torch.int32, device=dev, generator=g)
    for t in range(200):
        env.step(acts[t % 100], sync_edges=False)
    torch.cuda.synchronize()
    out = {"config": f"{a.agents}x{a.envs}", "one_launch": os.environ.get("GSM_EAGER_ONE_LAUNCH", "0")}
    for name, fn in (("env_step", lambda t: env.step(acts[t % 100], sync_edges=False)),):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(a.steps):
            fn(t)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name + "_host_us"] = (t1 - t0) / a.steps * 1e6
        out[name + "_device_us"] = (t2 - t0) / a.steps * 1e6
    # bare C-ABI calls: the wrapper's own cost left out
    lib, h = env.lib, env._h
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    ptrs = [C.c_void_p(acts[t].data_ptr()) for t in range(100)]
    fmt = _lib.ACT_INDEX
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.steps):
        lib.gsm_step(h, ptrs[t % 100], fmt, st)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["abi_host_us"] = (t1 - t0) / a.steps * 1e6
    out["abi_device_us"] = (t2 - t0) / a.steps * 1e6
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
