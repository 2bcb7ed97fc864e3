"""Where does the fixed cost of one short rollout replay go? The driver's bench
line times ONE replay of a 20-step graph from an idle GPU (barrier +
synchronize on both sides); back-to-back replays cost less per step.

Measures (µs, medians over R repetitions, each from idle):
  sync_only     torch.cuda.synchronize() with nothing queued (host round trip)
  tiny_op       a 1-element torch add + synchronize (launch + completion floor)
  roll1         replay of a 1-step rollout graph + synchronize
  rollK         replay of a K-step rollout graph + synchronize
  rollK_kernel  the K-step rollout kernel's own duration in that replay (HIP
                events recorded on the stream around the replay call)
  rollK_b2b     per replay, R replays back to back (one synchronize)
Run it per library build (GSM_LIB_PATH) to compare launch paths.

Usage: python tools/probe_launch.py [--K 20] [--R 15] [--N 24] [--B 8192]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gs-marl_amd")]

import torch  # noqa: E402

from gsmarl_amd import EnvConfig, GpuBatchEnv  # noqa: E402


def med(xs):
    return round(statistics.median(xs), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--R", type=int, default=15)
    ap.add_argument("--N", type=int, default=24)
    ap.add_argument("--B", type=int, default=8192)
    # host wait mode of synchronize: HIP's hipSetDeviceFlags schedule flag,
    # set before (early) or after (late) the first GPU use
    ap.add_argument("--sched", choices=["default", "spin", "yield", "block"], default="default")
    ap.add_argument("--sched-when", choices=["early", "late"], default="early")
    a = ap.parse_args()
    flag = {"spin": 1, "yield": 2, "block": 4}.get(a.sched)
    if flag and a.sched_when == "early":
        import ctypes
        print("hipSetDeviceFlags", ctypes.CDLL("libamdhip64.so.7").hipSetDeviceFlags(flag), file=sys.stderr)
    dev = torch.device("cuda", 0)
    env = GpuBatchEnv(EnvConfig(n_agents=a.N, n_envs=a.B, seed=1234), dev)
    acts = torch.randint(0, 5, (100, a.B, a.N), dtype=torch.int32, device=dev)
    env.reset(seed=1234, sync_edges=False)
    env.capture(acts, 1, slot=1, kernels="roll")
    env.capture(acts, a.K, slot=0, kernels="roll")
    x = torch.zeros(1, device=dev)
    if flag and a.sched_when == "late":
        import ctypes
        print("hipSetDeviceFlags", ctypes.CDLL("libamdhip64.so.7").hipSetDeviceFlags(flag), file=sys.stderr)
    for _ in range(3):   # first uses
        env.replay(1)
        env.replay(0)
        x.add_(1)
    torch.cuda.synchronize(dev)

    def wall(fn, R):
        out = []
        for _ in range(R):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            out.append((time.perf_counter() - t0) * 1e6)
        return out

    res = {"K": a.K, "N": a.N, "B": a.B, "lib": os.environ.get("GSM_LIB_PATH", "libgsm.so"),
           "sched": a.sched + ("/" + a.sched_when if flag else "")}
    res["sync_only_us"] = med(wall(lambda: None, a.R))
    # the host side of one replay call alone (returns before the kernel runs):
    # GpuBatchEnv.replay (Python, ctypes, current-stream lookup) and the bare
    # C call with the stream pointer cached
    import ctypes as C
    calls, bare = [], []
    sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(a.R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        env.replay(0)
        calls.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        env.lib.gsm_graph_launch(env._h, 0, sp)
        bare.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize(dev)
    res["replay_call_us"] = med(calls)
    res["bare_launch_call_us"] = med(bare)
    res["tiny_op_us"] = med(wall(lambda: x.add_(1), a.R))
    res["roll1_us"] = med(wall(lambda: env.replay(1), a.R))
    res[f"roll{a.K}_us"] = med(wall(lambda: env.replay(0), a.R))
    ev = []
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.R):
        torch.cuda.synchronize(dev)
        s.record()
        env.replay(0)
        e.record()
        torch.cuda.synchronize(dev)
        ev.append(s.elapsed_time(e) * 1e3)
    res[f"roll{a.K}_events_us"] = med(ev)
    torch.cuda.synchronize(dev)
    s.record()
    for _ in range(a.R):
        env.replay(0)
    e.record()
    torch.cuda.synchronize(dev)
    res[f"roll{a.K}_b2b_us"] = round(s.elapsed_time(e) * 1e3 / a.R, 2)
    # a 100-step launch (an episode): per step, events around one launch and
    # around back-to-back launches
    env.capture(acts, 100, slot=2, kernels="roll")
    env.replay(2)
    torch.cuda.synchronize(dev)
    ev = []
    for _ in range(max(3, a.R // 3)):
        torch.cuda.synchronize(dev)
        s.record()
        env.replay(2)
        e.record()
        torch.cuda.synchronize(dev)
        ev.append(s.elapsed_time(e) * 1e3 / 100)
    res["roll100_events_us_per_step"] = med(ev)
    s.record()
    for _ in range(5):
        env.replay(2)
    e.record()
    torch.cuda.synchronize(dev)
    res["roll100_b2b_us_per_step"] = round(s.elapsed_time(e) * 1e3 / 500, 3)
    # the 20-step graph across an episode boundary (every env auto-resets at
    # step 100: the driver's bench line holds one): advance to step 90 first
    env.capture(acts, 90, slot=1, kernels="roll")
    wb, eb = [], []
    for _ in range(max(3, a.R // 3)):
        env.reset(seed=1234, sync_edges=False)
        env.replay(1)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        s.record()
        env.replay(0)
        e.record()
        torch.cuda.synchronize(dev)
        wb.append((time.perf_counter() - t0) * 1e6)
        eb.append(s.elapsed_time(e) * 1e3)
    res[f"roll{a.K}_boundary_us"] = med(wb)
    res[f"roll{a.K}_boundary_events_us"] = med(eb)
    # the bench's sequence: 5-step and 85-step graphs, then the timed 20-step
    # graph's FIRST replay (fresh capture each repetition) vs its later ones
    first, later = [], []
    for rep in range(4):
        env.capture(acts, 5, slot=2, kernels="roll")
        env.capture(acts, 85, slot=3, kernels="roll")
        env.capture(acts, a.K, slot=0, kernels="roll")
        for r2 in range(2):
            env.reset(seed=1234, sync_edges=False)
            env.replay(2)
            env.replay(3)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            env.replay(0)
            torch.cuda.synchronize(dev)
            (first if r2 == 0 else later).append((time.perf_counter() - t0) * 1e6)
    res[f"roll{a.K}_bench_seq_first_us"] = med(first)
    res[f"roll{a.K}_bench_seq_second_us"] = med(later)
    res["gave_up"] = bool(env.roll_gave_up())
    print(json.dumps(res), flush=True)
    env.close()


if __name__ == "__main__":
    main()
