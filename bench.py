#!/usr/bin/env python3
"""Throughput bench of the batched MultiAgentGraphConstrainEnv step path.

Metric (BASELINE.json): agent-steps/sec, cooperative navigation, 24 agents x
8192 envs per MI355X (the headline config; N GPUs = weak scaling, each rank
owns 8192 envs with global Philox env ids, BASELINE configs[4] at N=8).

A "step" = one env.step of every env on the GPU: action force, pairwise
contact physics, integration, reward, collision cost, done/auto-reset, node
features and the packed COO edge list (inside a graph the
segmented configs run one launch per step — step j+1's kernel first emits
step j's edges — plus one emit launch at the end of the graph). Actions
are pre-generated on device (100 x B x N int32, uniform over the 5 discrete
actions) so the timed region has no host work; the K timed steps are
replayed from HIP graphs of one episode (100 steps) each, with the per-episode
RCCL all-reduce of episode metrics between chunks when N > 1.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
Prints ONE JSON line on rank 0 (diagnostics go to stderr).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gs-marl_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "agent-steps/sec, coop-navigation 24 agents × 8192 envs, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def step_kernel_bytes(B, N, No, EL, action_bytes, seg=True, envs_per_block=None):
    """Algorithmic HBM bytes of one step-kernel launch.

    Segmented path (M = N + No <= 64): per env, reads pos of every entity,
    agent vel, actions, the 16-B counters, the agent contact-candidate masks
    and the cached obstacle adjacency rows; writes agent pos/vel, the agent
    node-feature rows (goal/obstacle rows are static within an episode), reward,
    cost, the new masks, counters, done, edge count and the per-block edge sum.
    Re-layout at episode end rewrites goal/obstacle pos and static node rows:
    amortised over the episode length. Tile path (M > 64): the same with
    W = ceil(M/64) mask words per row; obstacle rows re-read their
    obstacle-only words and rewrite the chunks holding agent columns; agent
    node-feature rows are 6 floats per step (the type column is static)."""
    E, M = 2 * N + No, N + No
    if seg:
        reads = 8 * E + 8 * N + action_bytes * N + 16 + 8 * N + 8 * No
        writes = 8 * N + 8 * N + 28 * N + 4 * N + 4 * N + 8 * N + 8 * M + 16 + 1 + 4
        reset = (8 * (E - N) + 28 * (E - N) + 8) / EL
        per_block = envs_per_block or 4 * min(64 // M, 4)   # gsm_sizes.envs_per_block
    else:
        W, ka = (M + 63) // 64, (N + 63) // 64
        reads = 8 * E + 8 * N + action_bytes * N + 16 + 8 * N * W + 8 * No * (W - ka)
        writes = 8 * N + 8 * N + 24 * N + 4 * N + 4 * N + 8 * N * W + 8 * (N * W + No * ka) + 16 + 1 + 4
        reset = (8 * (E - N) + 28 * (E - N) + 4 * N + 8) / EL
        per_block = 1
    return B * (reads + writes + reset + 4 / per_block)


def emit_kernel_bytes(B, N, No, total_edges, seg=True):
    """Algorithmic HBM bytes of one edge-emit launch: entity positions, the
    adjacency row masks (W = ceil(M/64) words per collider row on the tile
    path, 1 on the segmented path), the env's edge count, the int64 edge_ptr
    entry and 12 B per edge (src, dst int32 + fp32 distance)."""
    E, M = 2 * N + No, N + No
    per_env = 8 * E + 4 + 8 + 8 * M * (1 if seg else (M + 63) // 64)
    return B * per_env + 12 * total_edges


def lag_extra_bytes(B, N, No, total_edges, seg=True):
    """Bytes a lagged step kernel moves on top of step_kernel_bytes: the
    previous step's emission minus what the step part already reads (entity
    positions, the obstacle rows' cached words) — the rest of the row masks,
    the env's edge sum, the edge_ptr entry and 12 B per edge."""
    M = N + No
    if seg:
        masks = 8 * N
    else:
        W, ka = (M + 63) // 64, (N + 63) // 64
        masks = 8 * (M * W - No * (W - ka))
    return B * (masks + 4 + 8) + 12 * total_edges


def ragged_kernel_bytes(env, EL, action_bytes, total_edges):
    """Algorithmic HBM bytes of one ragged step / emit launch, summed over the
    batch's actual env shapes (N_env agents, T targets, M colliders).

    step: reads collider + target positions, agent vel, actions, counters and
    the shape word; writes agent pos/vel, 6 node-feature floats per agent,
    reward/cost/assign (N_max each), the M row masks, counters, done, edge
    count; re-layout (all E_max rows of pos and node features, N_max vel)
    amortised over the episode. emit: reads all E_max positions, the M row
    masks, edge count and shape; writes edge_ptr and 12 B per edge."""
    import numpy as np
    sh = env.t["env_shape"].cpu().numpy()
    n, scn = (sh & 0xFF).astype(np.int64), sh >> 8
    T = np.where(scn == 0, n, np.where(scn == 1, 1, 2))
    M = n + np.where(scn == 0, n, 0)
    Nmax, Emax = env.N, env.E
    reads = 8 * (M + T) + 8 * n + action_bytes * n + 16 + 4
    writes = 8 * n + 8 * n + 24 * n + 12 * Nmax + 8 * M + 16 + 1 + 4
    reset = (8 * Emax + 28 * Emax + 8 * Nmax + 4) / EL
    step = float((reads + writes + reset).sum()) + 4 * len(n) / 4
    emit = float((8 * Emax + 8 * M + 4 + 4 + 8).sum()) + 12 * total_edges
    return step, emit


CONFIGS = {   # BASELINE.json configs runnable as a one-GPU bench line
    "h": dict(scenario="navigation", n_agents=24, n_envs=8192, desc="BASELINE headline / configs[4] shard"),
    "c2": dict(scenario="navigation", n_agents=3, n_envs=4096, desc="BASELINE configs[1]"),
    "c3": dict(scenario="navigation", n_agents=96, n_envs=1024, desc="BASELINE configs[2]"),
    "c4": dict(scenario="mixed", n_agents=24, n_envs=8192, n_agents_min=3,
               desc="BASELINE configs[3]: mixed navigation/polygon/line, N_env in {3..24}"),
}


def _cpu_worker(job):
    """One host process: step one CPU restatement for `seconds`; returns
    (agent-steps, elapsed). kind "nav": oracle/mpe_ref.py (object-per-entity
    MPE, Python pair loop, fp64), one env; kind "ragged": oracle/ragged_ref.py
    over a 30-env mixed sample (per-env NumPy + the assignment restatement)."""
    kind, cfgd, seconds, seed = job
    import numpy as np
    sys.path.insert(0, str(ROOT))
    rng = np.random.default_rng(seed)
    steps, agents = 0, 0
    if kind == "nav":
        from oracle import mpe_ref
        from oracle.batch_ref import make_cfg
        n = cfgd["n_agents"]
        env = mpe_ref.GraphConstrainEnv(make_cfg(n_agents=n, seed=seed))
        env.reset(seed=seed)
        eye = np.eye(5)
        agents = n
        t0 = time.perf_counter()
        while True:
            env.step(list(eye[rng.integers(0, 5, size=n)]))
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    else:
        from oracle import ragged_ref as rr
        keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
        rcfg = rr.make_cfg(**{k: v for k, v in cfgd.items() if k in keys})
        rcfg.n_envs, rcfg.env_base = 30, 30 * seed
        st = rr.new_state(rcfg)
        agents = int(st["n"].sum())
        t0 = time.perf_counter()
        while True:
            st, _ = rr.step(rcfg, st, rng.integers(0, 5, (30, cfgd["n_agents"])), 1, np.float64)
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return steps * agents, el


def cpu_baseline(cfg, seconds, cores):
    """The CPU restatement of the reference path timed on `cores` host
    processes (one env or env sample per process, like the reference's
    subprocess vec-env); the reference's own CPU path is absent
    (readme.md:1), so this is a port. Returns the all-core rate and the mean
    single-process rate."""
    import multiprocessing as mp
    kind = "ragged" if cfg.ragged else "nav"
    cfgd = cfg.to_dict()
    jobs = [(kind, cfgd, seconds, 1000 + i) for i in range(cores)]
    if cores == 1:
        res = [_cpu_worker(jobs[0])]
    else:
        # spawned children: fresh interpreters that never touch the GPU
        with mp.get_context("spawn").Pool(cores) as pool:
            res = pool.map(_cpu_worker, jobs)
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    single = sum(r[0] / r[1] for r in res) / len(res)
    what = ("oracle/mpe_ref.py GraphConstrainEnv.step (object-per-entity MPE restatement, fp64, Python "
            f"pair loop), N={cfg.n_agents}, one env per process") if kind == "nav" else (
            "oracle/ragged_ref.py step over a 30-env mixed sample per process (per-env NumPy, fp64, "
            "assignment via oracle/lsa_ref.py)")
    return dict(value=total / wall, unit="agent-steps/s", cores=cores, kind="port",
                single_core_value=single,
                sample=f"{cores} host processes x {seconds:.0f} s of {what}; the reference's own CPU path is "
                       f"absent (readme.md:1)")


def host_cores():
    """The host-core share of this job: the affinity set, capped at 16 (the
    GPU box's share per GPU; nproc shows the whole machine there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def pmc_traffic(key):
    """HBM bytes per step-kernel launch from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, written by tools/pmc_traffic.py)."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="h",
                    help="BASELINE config (h = 24 agents x 8192 envs per GPU)")
    ap.add_argument("--n-agents", type=int, default=None, help="override the config's agents")
    ap.add_argument("--n-envs", type=int, default=None, help="override the config's envs per GPU")
    ap.add_argument("--kernel-launches", type=int, default=100,
                    help="back-to-back launches per kernel for the event-timed roofline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-cores", type=int, default=0, help="host processes for the CPU baseline (0: all, <= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="skip the roofline timing (null)")
    ap.add_argument("--eager", action="store_true", help="launch steps eagerly instead of HIP graphs")
    ap.add_argument("--unfused", action="store_true",
                    help="two launches per step in the graphs (no lagged emission)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from gsmarl_amd import EnvConfig, GpuBatchEnv
    from gsmarl_amd.distributed import all_reduce_metrics, max_over_ranks, shard_config

    spec = dict(CONFIGS[args.config])
    cfg_name = spec.pop("desc")
    if args.n_agents:
        spec["n_agents"] = args.n_agents
    if args.n_envs:
        spec["n_envs"] = args.n_envs
    N, B = spec["n_agents"], spec["n_envs"]
    cfg = shard_config(EnvConfig(seed=1234, **spec), rank, world)
    env = GpuBatchEnv(cfg, dev)
    EL = cfg.episode_length
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    actions = torch.randint(0, 5, (EL, B, N), dtype=torch.int32, device=dev, generator=gen)
    env.reset(seed=cfg.seed, sync_edges=False)

    K, W = args.steps, args.warmup
    chunk = min(K, EL)
    n_chunks, rem = divmod(K, chunk)
    gk = "unfused" if args.unfused else "both"
    if not args.eager:
        if W > 0:
            env.capture(actions, W, timing=False, slot=2, kernels=gk)
        env.capture(actions, chunk, timing=False, slot=0, kernels=gk)
        if rem:
            env.capture(actions, rem, timing=False, slot=1, kernels=gk)
    # warmup
    if W > 0:
        if args.eager:
            for t in range(W):
                env.step(actions[t % EL], sync_edges=False)
        else:
            env.replay(2)
    torch.cuda.synchronize()
    metrics = torch.zeros(3, dtype=torch.float64, device=dev)

    def run_chunk(n, slot):
        if args.eager:
            for t in range(n):
                env.step(actions[t % EL], sync_edges=False)
        else:
            env.replay(slot)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_chunks):
        run_chunk(chunk, 0)
        if world > 1:   # the only collective: per-episode metrics (RCCL/xGMI)
            metrics.copy_(env.episode_metrics())
            all_reduce_metrics(metrics)
    if rem:
        run_chunk(rem, 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, device=dev) if world > 1 else elapsed

    total_edges = int(env.t["edge_ptr"][B].item())
    seg_cfg = (N + cfg.n_obstacles) <= 64 and not cfg.ragged
    # agents per step on this rank (ragged: sum of N_env), summed over ranks
    agents = int((env.t["env_shape"] & 0xFF).sum().item()) if cfg.ragged else B * N
    if world > 1:
        agents = int(all_reduce_metrics(torch.tensor([float(agents), 0.0, 0.0], dtype=torch.float64,
                                                     device=dev))[0].item())
    value = agents * K / elapsed
    ms_per_step = elapsed / K * 1e3

    # Roofline: each kernel's mean launch duration, HIP events (graph event
    # nodes on the launch stream) around L back-to-back launches of that
    # kernel alone, after the timed region. Event nodes between kernels would
    # add their own packet time to every launch.
    roofline = None
    if not args.no_kernel_timing and not args.eager:
        L = args.kernel_launches
        seg = (N + cfg.n_obstacles) <= 64 and not cfg.ragged
        lag = seg and not args.unfused
        env.capture(actions, L, slot=3, kernels="lag" if lag else "step", time_ends=True)
        env.replay(3)
        torch.cuda.synchronize()
        step_ms = env.graph_kernel_ms(3)[0]
        env.capture(None, L, slot=3, kernels="emit", time_ends=True)
        env.replay(3)
        torch.cuda.synchronize()
        emit_ms = env.graph_kernel_ms(3)[1]
        edges_now = int(env.t["edge_ptr"][B].item())
        if cfg.ragged:
            sb, eb = ragged_kernel_bytes(env, EL, 4, edges_now)
            names = ("gsm_step_ragged_kernel", "gsm_emit_ragged_kernel")
        else:
            sb = step_kernel_bytes(B, N, cfg.n_obstacles, EL, 4, seg, env.sizes.envs_per_block)
            if lag:
                sb += lag_extra_bytes(B, N, cfg.n_obstacles, edges_now, seg)
            eb = emit_kernel_bytes(B, N, cfg.n_obstacles, edges_now, seg)
            fam = "seg" if seg else "tile"
            names = (f"gsm_step_{fam}_kernel" + ("<lagged emission>" if lag else ""), f"gsm_emit_{fam}_kernel")
        kern = {"step": dict(kernel=names[0], ms=step_ms, bytes=sb, gbs=sb / (step_ms * 1e-3) / 1e9),
                "emit": dict(kernel=names[1], ms=emit_ms, bytes=eb, gbs=eb / (emit_ms * 1e-3) / 1e9)}
        # a lagged chain runs the emit kernel once per graph, the step kernel every step
        dom = "step" if (lag or step_ms >= emit_ms) else "emit"
        k = kern[dom]
        other = kern["emit" if dom == "step" else "step"]
        roofline = dict(kernel=k["kernel"], bound="hbm", achieved=round(k["gbs"], 1), peak=HBM_PEAK_GBS,
                        unit="GB/s", frac=round(k["gbs"] / HBM_PEAK_GBS, 4),
                        traffic=pmc_traffic(f"{'lag' if (lag and dom == 'step') else dom}:{cfg.scenario}:N{N}:B{B}"),
                        algorithmic_bytes_per_launch=int(k["bytes"]), mean_launch_us=round(k["ms"] * 1e3, 3),
                        timing=f"HIP events around {L} back-to-back graph launches of the kernel",
                        other_kernel=dict(kernel=other["kernel"], achieved=round(other["gbs"], 1),
                                          algorithmic_bytes_per_launch=int(other["bytes"]),
                                          mean_launch_us=round(other["ms"] * 1e3, 3)))
        log(f"kernels: {json.dumps(kern)}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_seconds, args.cpu_cores or host_cores())

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "agent-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: Philox4x32-10 layouts, uniform random discrete actions pre-generated on device",
            "config": {"workload": (f"cooperative_navigation {N} agents x {B} envs per GPU "
                                    f"({N} goals, {cfg.n_obstacles} obstacles; {cfg_name})") if not cfg.ragged
                       else f"{cfg.scenario} up to {N} agents x {B} envs per GPU ({cfg_name})",
                       "scenario": cfg.scenario, "n_agents": N, "n_envs_per_gpu": B, "global_envs": world * B,
                       "agents_per_step": agents,
                       "episode_length": EL, "mean_edges_per_env": round(total_edges / B, 2),
                       "parallelism": f"env-sharded x{world} (no data-path collective)",
                       "launch": "eager" if args.eager else ("hip-graph per 100-step episode" + (
                           ", lagged emission (one launch per step)" if (seg_cfg and not args.unfused)
                           else ", step + emit launch per step"))},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
