#!/usr/bin/env python3
"""Throughput bench of the batched MultiAgentGraphConstrainEnv step path.

Metric (BASELINE.json): agent-steps/sec, cooperative navigation, 24 agents x
8192 envs per MI355X (the headline config; N GPUs = weak scaling, each rank
owns 8192 envs with global Philox env ids, BASELINE configs[4] at N=8).

A "step" = one env.step of every env on the GPU: action force, pairwise
contact physics, integration, reward, collision cost, done/auto-reset, node
features and the packed COO edge list; every observation output of every step
is written to HBM. Inside a graph every BASELINE config runs
all steps of the episode graph in ONE fused rollout launch (GSM_GRAPH_ROLL:
env state kept on chip, the CSR prefix handed between workgroups in-launch;
the headline and N = 6 / 12 one env per wave, C2 four envs per wave, C3 one
workgroup per env, C4 the ragged rollout); other shapes run one launch per
step (step j+1's kernel first emits step j's edges); `--no-roll` /
`--unfused` select those chains instead. `--eager` times env.step calls,
`--policy` / `--policy-graph` a closed loop with a trivial policy (eager, or
policy + step captured in one torch CUDA graph), `--buffer` the rollout
buffer (every step into its own slot). Actions are pre-generated on device
(100 x B x N int32, uniform over the 5 discrete actions) so the timed region
has no host work; the K timed steps are replayed from HIP graphs of one
episode (100 steps) each; when N > 1 the ranks' shards need no exchange,
and the RCCL all-reduce of the episode metrics runs after the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
Prints ONE JSON line on rank 0 (diagnostics go to stderr).
"""
from __future__ import annotations

import argparse
import gc
import json
import math
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


def roll_step_bytes(B, N, No, EL, action_bytes, total_edges, seg=True):
    """Algorithmic HBM bytes per step of the fused rollout launch. The
    simulator state (positions, velocities, masks, counters) stays on chip and
    is loaded / stored once per launch (left out: under 1% over 100 steps); a
    step reads its actions and writes its observation outputs: the agent
    node-feature rows (7 floats on the segmented path, 6 on the tile path
    whose type column is static), reward, cost, done, and (one iteration
    later) the edge_ptr entry and 12 B per edge; at an episode end the static
    node rows, amortised over the episode. (The tile path also re-reads its
    contact words and the previous step's row masks from L2: on-chip traffic
    of the workgroup's own writes, not counted.)"""
    E = 2 * N + No
    writes = (28 if seg else 24) * N + 4 * N + 4 * N + 1 + 8
    reset = (28 * (E - N) + 8) / EL
    return B * (action_bytes * N + writes + reset) + 12 * total_edges


def survey_bytes_per_agent_step(N, No, action_bytes, total_edges, B):
    """SURVEY.md §8(d)'s algorithmic bytes per agent-step, the per-unit figure
    the contract prices a whole step at: B_as = 32 (pos+vel read+write) + A
    (action) + 8 (own goal) + 8·No/N (obstacle positions) + 9 (reward, cost,
    done) + (E/N)·F·4 (node table, F = 7) + 12·ē (edges per agent: int32 src,
    dst + fp32 distance), ē measured."""
    E = 2 * N + No
    ebar = total_edges / (B * N)
    return 32 + action_bytes + 8 + 8 * No / N + 9 + (E / N) * 7 * 4 + 12 * ebar


def ragged_kernel_bytes(env, EL, action_bytes, total_edges):
    """Algorithmic HBM bytes of one ragged step / emit launch, summed over the
    batch's actual env shapes (N_env agents, T targets, M colliders).

    step: reads collider + target positions, agent vel, actions, counters and
    the shape word; writes agent pos/vel, 6 node-feature floats per agent,
    reward/cost/assign (N_max each), the M row masks, counters, done, edge
    count; re-layout (all E_max rows of pos and node features, N_max vel)
    amortised over the episode; polygon/line envs also read and write their
    assignment warm-start state (f64 column dual + int32 matching per agent,
    when the warm start is on). emit: reads all E_max positions, the M row
    masks, edge count and shape; writes edge_ptr and 12 B per edge. lag: what
    a lagged step kernel adds to the step (the emission less the collider and
    target positions and the shape word the step reads anyway)."""
    import numpy as np
    sh = env.t["env_shape"].cpu().numpy()
    n, scn = (sh & 0xFF).astype(np.int64), sh >> 8
    T = np.where(scn == 0, n, np.where(scn == 1, 1, 2))
    M = n + np.where(scn == 0, n, 0)
    Nmax, Emax = env.N, env.E
    reads = 8 * (M + T) + 8 * n + action_bytes * n + 16 + 4
    writes = 8 * n + 8 * n + 24 * n + 12 * Nmax + 8 * M + 16 + 1 + 4
    reset = (8 * Emax + 28 * Emax + 8 * Nmax + 4) / EL
    warm = np.where(scn != 0, 2 * 12 * n, 0) if env.cfg.lsa_warm_start else 0
    step = float((reads + writes + reset + warm).sum()) + 4 * len(n) / 4
    emit = float((8 * Emax + 8 * M + 4 + 4 + 8).sum()) + 12 * total_edges
    lag = emit - float((8 * (M + T) + 4).sum())
    return step, emit, lag


def ragged_roll_step_bytes(env, EL, action_bytes, total_edges):
    """Algorithmic HBM bytes per step of the ragged fused rollout launch,
    summed over the batch's env shapes: the step's actions and observation
    outputs (6 node-feature floats per agent, reward / cost / assign over
    N_max, done, the edge_ptr entry, 12 B per edge), the assignment's
    warm-start state of polygon/line envs (f64 column dual + int32 matching
    per agent, read and written), the static node rows of a reset amortised
    over the episode. The simulator state stays on chip (loaded / stored once
    per launch, left out); the per-env edge slabs the launch packs from are
    its own staging, not algorithmic traffic."""
    import numpy as np
    sh = env.t["env_shape"].cpu().numpy()
    n, scn = (sh & 0xFF).astype(np.int64), sh >> 8
    Nmax, Emax = env.N, env.E
    per = action_bytes * n + 24 * n + 12 * Nmax + 1 + 8 + (28 * Emax + 4) / EL
    warm = np.where(scn != 0, 2 * 12 * n, 0) if env.cfg.lsa_warm_start else 0
    return float((per + warm).sum()) + 12 * total_edges


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
    host = machine_cores()
    return dict(value=total / wall, unit="agent-steps/s", cores=cores, kind="port",
                single_core_value=single, cpu_model=cpu_model(),
                all_core=dict(value=single * host, cores=host,
                              how=f"extrapolated: the measured mean single-process rate x the host's {host} "
                                  "hardware threads (processes are independent envs with no shared state; a run "
                                  "on every host core would take the other GPUs' jobs' share of the box, whose "
                                  f"per-GPU share is the {cores} processes measured)"),
                sample=f"{cores} host processes x {seconds:.0f} s of {what}; the reference's own CPU path is "
                       f"absent (readme.md:1)")


def machine_cores():
    """Hardware threads of the whole host (os.cpu_count: every CPU of the
    machine, beyond this job's share)."""
    return os.cpu_count() or 1


def host_cores():
    """The host-core share of this job: the affinity set, capped at 16 (the
    GPU box's share per GPU; nproc shows the whole machine there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def code_object_hash(lib_path=None):
    """Hash of the gfx950 device code the bench runs: the `.hip_fatbin`
    section of the built libgsm.so (the offload bundle of every kernel). PMC
    figures are injected into a bench line only when they were collected on
    exactly this code (tools/pmc_traffic.py records the hash); edits to host
    code, comments or tools leave it unchanged."""
    import hashlib
    import struct
    if lib_path is None:
        from gsmarl_amd import _lib
        lib_path = _lib.LIB_PATH
    data = Path(lib_path).read_bytes()
    # ELF64 little-endian: section headers, then the section-name string table
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sec(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise RuntimeError(f"{lib_path}: no .hip_fatbin section")


PMC_FILE = ROOT / "profiles" / "pmc_kernels.json"
# What binds a kernel, from its PMC counters. Issue ceilings
# measured on MI355X (tools/probe_issue.hip, profiles/r4_probe_issue.txt:
# every CU at 8 waves per SIMD, independent instructions): a SIMD issues at
# most 0.447 wave64 VALU instructions per shader cycle, and a CU at most
# 0.934 SALU instructions per cycle in total — the scalar unit is shared by
# the CU's four SIMDs (2 waves per SIMD already saturate it), and VALU
# instructions that write an SGPR (v_readlane) draw on the same budget. The
# launch's own cycle count is GRBM_GUI_ACTIVE / 8 (the counter sums the 8
# XCDs), so the fractions below are ratios within one profiled run and do not
# depend on the bench's timing or clock.
VALU_PEAK = 0.447     # wave64 VALU instructions per SIMD and shader cycle
SALU_PEAK = 0.934     # SALU instructions per CU and shader cycle
N_SIMDS = 1024        # 256 CUs x 4 SIMDs
N_CUS = 256
N_XCDS = 8
BOUND_AT = 0.6        # a pipe (or HBM) above this share of its ceiling binds; none: latency-bound


def pmc_entry(key):
    """(entry, note) for kernel `key` from profiles/pmc_kernels.json: HBM
    bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) and
    VALU/SALU instructions per launch. None when absent or collected on
    another build of the device code (stale figures are never used)."""
    if not PMC_FILE.exists():
        return None, "no profiles/pmc_kernels.json"
    try:
        d = json.loads(PMC_FILE.read_text())
    except Exception as e:   # a broken file must not break the bench line
        return None, f"unreadable pmc file: {e}"
    if d.get("code_object_hash") != code_object_hash():
        return None, "stale: profiles/pmc_kernels.json was collected on another build of the kernels"
    e = d.get("entries", {}).get(key)
    return (e, "ok") if e else (None, f"no PMC entry for {key}")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); without torchrun bench.py spawns one process per GPU itself")
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
    ap.add_argument("--settle-ms", type=float, default=20.0,
                    help="before the warmup, whole untimed episodes (EL steps each, so the alignment holds) "
                         "until this much wall time has passed with the GPU busy: clocks at their loaded level "
                         "(the driver's 20-step line: 11.5-11.6 us/step without, 10.85 with 20 ms; DESIGN.md §8)")
    ap.add_argument("--no-align", action="store_true",
                    help="do not advance (untimed) so that the timed region contains an episode boundary")
    ap.add_argument("--eager", action="store_true", help="launch steps eagerly instead of HIP graphs")
    ap.add_argument("--policy", action="store_true",
                    help="closed loop: GpuGraphVecEnv(output='torch', graph='coo').step() with an on-device "
                         "greedy policy reading each step's obs (the runner's path; context, not the headline)")
    ap.add_argument("--policy-graph", action="store_true",
                    help="the closed loop of --policy with the policy and env.step captured into one "
                         "torch.cuda graph per step (replayed every step)")
    ap.add_argument("--policy-graph-steps", type=int, default=1,
                    help="--policy-graph: steps of policy + env.step captured in the one graph (a runner "
                         "collecting a rollout on device replays one graph per S steps)")
    ap.add_argument("--policy-act", choices=("index", "cont"), default="index",
                    help="--policy / --policy-graph action format: index = the greedy discrete action (int32, "
                         "three small kernels), cont = the continuous bang-bang action sign(goal - position) "
                         "(one kernel)")
    ap.add_argument("--vec-env", choices=("numpy-dense", "numpy-coo"), default=None,
                    help="the MAPPO runner's host surface: GpuGraphVecEnv(output='numpy', graph=dense|coo)"
                         ".step(host actions) per step, every returned array on the host (make_train_env's "
                         "default is numpy-dense); context, not the headline")
    ap.add_argument("--unfused", action="store_true",
                    help="two launches per step in the graphs (no lagged emission)")
    ap.add_argument("--no-roll", action="store_true",
                    help="one launch per step (lagged chain) even where a fused rollout launch exists")
    ap.add_argument("--buffer", action="store_true",
                    help="the training consumer: every step written to its own slot of a GraphRolloutBuffer "
                         "(gsm_graph_capture_into: one rollout launch per episode, step k's outputs in slot k+1)")
    # launcher self-test only (tests/test_bench_launcher.py): a CPU stand-in env
    # module and gloo; the line it prints is marked as not a measurement
    ap.add_argument("--selftest-env", default=None, help=argparse.SUPPRESS)
    # test only (tests/test_gpu_bench_rccl.py): join a process group of one
    # rank and run every collective of the multi-GPU path on one GPU
    ap.add_argument("--force-pg", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def align_steps(warmup, steps, EL):
    """Untimed steps after warmup so that the timed region [P, P+K) holds an
    episode boundary (every env auto-resets when its step count reaches EL,
    and all envs start together): P = EL - ceil(K/2) (mod EL)."""
    return (EL - (steps + 1) // 2 - warmup) % EL


def boundaries_in(p, k, EL):
    """Episode boundaries (auto-resets) inside steps p+1 .. p+k."""
    return (p + k) // EL - p // EL


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned_rank(argv, rank, world, port):
    """Entry of one spawned rank (a fresh interpreter: nothing touched the GPU
    in it yet)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rc = run_rank(parse_args(argv))
    if rc:
        sys.exit(rc)


def launch_ranks(args, argv):
    """`bench.py --gpus N` without torchrun: one spawned process per GPU (the
    parent never initialises the GPU — torch.cuda.device_count() does not on
    this image), each joining an RCCL process group; fails (non-zero) when
    fewer than N GPUs are visible or any rank fails, never falls back to fewer
    ranks."""
    import multiprocessing as mp
    n = args.gpus
    if args.selftest_env is None:
        import torch
        have = torch.cuda.device_count()
        if have < n:
            log(f"error: --gpus {n} but only {have} GPU(s) visible")
            return 3
    port = free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_spawned_rank, args=(argv, r, n, port)) for r in range(n)]
    for p in procs:
        p.start()
    rc = 0
    for p in procs:
        p.join()
        if p.exitcode != 0:
            log(f"error: rank {procs.index(p)} exited with {p.exitcode}")
            rc = rc or 1
            for q in procs:   # a failed rank leaves the others blocked in a collective
                if q.is_alive():
                    q.terminate()
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus > 1:
            return launch_ranks(args, argv)
        return run_rank(args)
    if int(ws) != args.gpus:
        log(f"error: WORLD_SIZE={ws} but --gpus={args.gpus}")
        return 2
    return run_rank(args)


def run_rank(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    stub = args.selftest_env is not None
    if stub:
        import importlib
        dev = torch.device("cpu")
        make_env = importlib.import_module(args.selftest_env).make_env

        def sync():
            pass
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

        def make_env(cfg, device):
            from gsmarl_amd import GpuBatchEnv
            return GpuBatchEnv(cfg, device)

        def sync():
            torch.cuda.synchronize(dev)
    pg = world > 1 or args.force_pg   # the collectives of the multi-GPU path run
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(free_port())
        if stub:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:   # RCCL over xGMI
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from gsmarl_amd import EnvConfig
    from gsmarl_amd.distributed import all_reduce_metrics, shard_config

    spec = dict(CONFIGS[args.config])
    cfg_name = spec.pop("desc")
    if args.n_agents:
        spec["n_agents"] = args.n_agents
    if args.n_envs:
        spec["n_envs"] = args.n_envs
    N, B = spec["n_agents"], spec["n_envs"]
    cfg = shard_config(EnvConfig(seed=1234, **spec), rank, world)
    venv = None
    if args.policy_graph:
        args.policy = True
    if args.vec_env and (args.policy or stub):
        log("error: --vec-env drives the host surface with pre-generated actions (no --policy)")
        return 2
    if (args.policy or args.vec_env) and not stub:
        # the vec-env a GS-MARL runner drives (gsmarl_amd/vec_env.py): on device
        # (--policy), or its host arrays (--vec-env)
        from gsmarl_amd.vec_env import GpuGraphVecEnv
        if args.vec_env:
            venv = GpuGraphVecEnv(cfg, dev, output="numpy", graph=args.vec_env.split("-")[1])
        else:
            venv = GpuGraphVecEnv(cfg, dev, output="torch", graph="coo")
        env = venv.batch
    else:
        env = make_env(cfg, dev)
    EL = cfg.episode_length
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    actions = torch.randint(0, 5, (EL, B, N), dtype=torch.int32, device=dev, generator=gen)
    env.reset(seed=cfg.seed, sync_edges=False)

    K, W = args.steps, args.warmup
    if args.buffer:   # whole episodes (one buffer replay = EL steps), the episode boundary at its end
        K = max(EL, -(-K // EL) * EL)
        W = -(-W // EL) * EL
        args.no_align = True
    A = 0 if args.no_align else align_steps(W, K, EL)
    chunk = min(K, EL)
    n_chunks, rem = divmod(K, chunk)
    gk = "unfused" if args.unfused else "both"
    eager = args.eager or args.policy or bool(args.vec_env)
    roll = not (args.unfused or args.no_roll or eager or stub)

    buf = None
    if args.buffer and not stub:
        # the rollout buffer a runner fills: slot 0 = the episode's first
        # observation, step k into slot k + 1 (every step at distinct addresses)
        from gsmarl_amd import GraphRolloutBuffer
        if args.eager or args.policy or args.vec_env or args.no_roll or args.unfused:
            log("error: --buffer replays the buffer's captured episode (no --eager/--policy/--no-roll/--unfused)")
            return 2
        buf = GraphRolloutBuffer(env, episode_length=EL)

    def capture(n, slot):
        """A graph of n steps: the fused rollout where the config has one
        (n >= 2), else the lagged / two-kernel chain. --buffer: the buffer's
        whole episode (EL steps into its slots) whatever n is."""
        nonlocal roll
        if buf is not None:
            buf.capture(actions, slot=slot)
            if not env.graph_is_rollout(slot):
                roll = False
            return
        if roll and n >= 2:
            try:
                env.capture(actions, n, timing=False, slot=slot, kernels="roll")
                return
            except Exception as e:   # GsmError: no rollout kernel for this config
                log(f"no fused rollout for this config ({e}); one launch per step")
                roll = False
        env.capture(actions, n, timing=False, slot=slot, kernels=gk)

    settle = args.settle_ms > 0 and not stub and buf is None   # (eager / closed loop: EL eager steps per pass)
    if buf is not None:
        buf.reset(seed=cfg.seed)
        capture(EL, 0)
    elif not eager:
        if W > 0:
            capture(W, 2)
        if settle:   # slot 3 holds a whole episode for the settle loop
            capture(EL, 3)
        elif A > 0:   # slot 3 is re-captured later by the roofline timing
            capture(A, 3)
        capture(chunk, 0)
        if rem:
            capture(rem, 1)
        elif settle and A > 0:   # the alignment in slot 1, captured before the settle loop
            capture(A, 1)

    obs = env.outputs()["obs"] if venv is not None and not args.vec_env else None

    # a trivial policy on device: the discrete action along the larger
    # component of (target - position) (obs[..., 4:6]; actions 1/2 = +x/-x,
    # 3/4 = +y/-y), as three kernels and no int64 scalar broadcasts: the
    # goal's bearing, its quadrant sector (int32 directly) and the sector's
    # action from a 5-entry table — the sectors in bearing order from -pi are
    # W, S, E, N, W
    sector_edges = torch.tensor([-0.75 * math.pi, -0.25 * math.pi, 0.25 * math.pi, 0.75 * math.pi],
                                dtype=torch.float32, device=dev)
    sector_action = torch.tensor([2, 4, 1, 3, 2], dtype=torch.int32, device=dev)

    def greedy(o):
        if args.policy_act == "cont":   # MPE continuous actions, u = a * sensitivity: one kernel
            return torch.sign(o[..., 4:6])
        return sector_action[torch.bucketize(torch.atan2(o[..., 5], o[..., 4]), sector_edges, out_int32=True)]

    pgraph = None
    if args.policy_graph and not stub:
        # policy + env.step of one step as one torch CUDA graph (gsm_step on a
        # capturing stream records the one-launch step where the config has
        # it: its hand-off epoch lives in device memory, so every replay
        # takes a fresh one; else the step + emit pair)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):   # warm the allocator and the policy's kernels (untimed steps)
                venv.step(greedy(obs))
        torch.cuda.current_stream().wait_stream(side)
        pgraph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(pgraph):
            for _ in range(args.policy_graph_steps):   # S steps of policy + env.step per replay
                venv.step(greedy(obs))   # obs: a view of the env's node features, static

    host_actions = actions.cpu().numpy() if args.vec_env else None
    vec_t = 0

    def run_steps(n, slot):
        nonlocal obs, vec_t
        if pgraph is not None:
            S = args.policy_graph_steps
            for t in range(n // S):
                pgraph.replay()
            for t in range(n % S):   # (a remainder: eager policy + step)
                venv.step(greedy(obs))
        elif host_actions is not None:
            # the runner's numpy loop: host actions in, host arrays and the
            # lazy infos out (each call returns after its host copies)
            for t in range(n):
                venv.step(host_actions[vec_t % EL])
                vec_t += 1
        elif venv is not None:
            for t in range(n):
                obs = venv.step(greedy(obs))[0]
        elif args.eager:
            for t in range(n):
                env.step(actions[t % EL], sync_edges=False)
        elif buf is not None:
            # the episode into the buffer's slots (the kernel launch of
            # GraphRolloutBuffer.replay; its host-side copy of the action
            # sequence into buf.actions is bookkeeping, left out)
            env.replay(0)
        else:
            env.replay(slot)

    # No collector pass inside the timed region (a full pass over torch's
    # object graph takes milliseconds; it would land in one step's time), and
    # none between the settle loop and the region either: milliseconds of an
    # idle GPU there let its clocks drop, and the 2-3 ms after them ran the
    # timed graphs slower — the h line 7.85 with the pass after the settle
    # loop, 7.00 us/step without it, same box (profiles/r5_ab/bench_gc/). So
    # everything that idles the GPU — the pass, the alignment's capture —
    # comes first, then the settle loop, the warmup, the alignment and the
    # region back to back.
    metrics = torch.zeros(3, dtype=torch.float64, device=dev)
    # ragged: the assignment warm start's certified / solved counters, read
    # around the timed region (outside it)
    lsa_stats = cfg.ragged and hasattr(env, "lsa_warm_stats")
    gc.collect()
    gc.disable()
    # settling (whole episodes: the alignment below still holds), warmup, then
    # the untimed alignment so the timed region holds an auto-reset
    settle_steps = 0
    a_slot = 1 if (settle and A > 0 and not rem) else 3
    if settle:
        # as many passes on every rank (the count for --settle-ms from the
        # first pass, the max over ranks), started together: the ranks reach
        # the region's barrier together instead of the early ones idling there
        # (and their clocks dropping, as above) for the startup skew
        sync()
        if pg:
            dist.barrier()
        run_steps(EL, 3)   # (the first pass runs cold: the count from the second)
        sync()
        t_s = time.perf_counter()
        run_steps(EL, 3)
        sync()
        settle_steps += 2 * EL
        passes = max(2, -(-int(args.settle_ms * 1e3) // max(1, int((time.perf_counter() - t_s) * 1e6))))
        if pg:
            pt = torch.tensor([passes], dtype=torch.int64, device=dev)
            dist.all_reduce(pt, op=dist.ReduceOp.MAX)
            passes = int(pt.item())
        for _ in range(passes - 2):
            run_steps(EL, 3)
            settle_steps += EL
            sync()
        if A > 0 and a_slot == 3:   # (slot 1 holds the remainder graph)
            capture(A, 3)
    for _ in range(W // EL if buf is not None else 0):
        run_steps(EL, 0)
    if W > 0 and buf is None:
        run_steps(W, 2)
    if A > 0:
        run_steps(A, a_slot)
    lsa0 = env.lsa_warm_stats() if lsa_stats else None
    # No collective inside the timed region but its barriers: the envs shard
    # with no exchange, and the episode-metric all-reduce (RCCL) runs once
    # after it. Beside a fused rollout, which fills every SIMD, an RCCL kernel
    # takes wave slots the rollout's grid needs and delays its workgroups:
    # one all-reduce per 100-step chunk overlapped with the chunks cost 7.44
    # vs 6.83 us per step at H (one rank, same box), and on several ranks the
    # kernel holds its slots until every peer arrives.
    bar_t = torch.zeros(1, dtype=torch.int32, device=dev)

    def region_barrier():
        """The region's closing synchronize + barrier: a one-element RCCL
        all-reduce queued behind the rank's work, then one synchronize — it
        completes on a rank only once every rank's contribution, queued behind
        that rank's graphs, has arrived. dist.barrier() (an all-reduce, then a
        device synchronize of its own) after a synchronize: 9.9-11.7 against
        8.9-9.2 us per step on the driver's 20-step line, one rank, same box
        (plain 8.6-8.9; profiles/r6_ab/bench_rccl/)."""
        if pg:
            dist.all_reduce(bar_t)
        sync()
    sync()
    if pg:
        dist.barrier()
    sync()
    # (diagnostic, GSM_BENCH_CHUNK_US=1: HIP events around every chunk of the
    # timed region, device times to stderr; event packets in the region)
    chunk_ev = ([torch.cuda.Event(enable_timing=True) for _ in range(n_chunks + 1)]
                if os.environ.get("GSM_BENCH_CHUNK_US") and not stub else None)
    t0 = time.perf_counter()
    if chunk_ev:
        chunk_ev[0].record()
    for ci in range(n_chunks):
        run_steps(chunk, 0)
        if chunk_ev:
            chunk_ev[ci + 1].record()
    if rem:
        run_steps(rem, 1)
    region_barrier()
    elapsed = time.perf_counter() - t0
    if chunk_ev:
        log("timed region chunks (device us): " + ", ".join(
            f"{chunk_ev[i].elapsed_time(chunk_ev[i + 1]) * 1e3:.1f}" for i in range(n_chunks))
            + f"; wall {elapsed * 1e6:.1f}")
    gc.enable()
    lsa1 = env.lsa_warm_stats() if lsa0 is not None else None

    # every rank's timed region; value uses the slowest (max over ranks)
    per_rank = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if pg:
        gathered = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(gathered, per_rank)
        times = [float(g.item()) for g in gathered]
    else:
        times = [elapsed]
    elapsed = max(times)
    # a bounded in-launch wait of a fused rollout that timed out leaves invalid
    # outputs: no measurement (decided on every rank together)
    bad = 1.0 if (roll and env.roll_gave_up()) else 0.0
    if pg:
        bad = float(all_reduce_metrics(torch.tensor([bad, 0.0, 0.0], dtype=torch.float64, device=dev))[0].item())
    if bad:
        log("ERROR: a fused rollout launch gave up waiting on a predecessor; no valid measurement")
        env.close()
        if pg:
            dist.destroy_process_group()
        return 3
    # the episode metrics over all ranks: the RCCL all-reduce (after the
    # timed region, see there)
    metrics.copy_(env.episode_metrics())
    all_reduce_metrics(metrics)
    ep_rew, ep_cost, episodes = (float(x) for x in metrics.cpu())

    total_edges = int(env.t["edge_ptr"][B].item())
    seg_cfg = (N + cfg.n_obstacles) <= 64 and not cfg.ragged
    # agents per step on this rank (ragged: sum of N_env), summed over ranks
    agents = int((env.t["env_shape"] & 0xFF).sum().item()) if cfg.ragged else B * N
    if pg:
        agents = int(all_reduce_metrics(torch.tensor([float(agents), 0.0, 0.0], dtype=torch.float64,
                                                     device=dev))[0].item())
    value = agents * K / elapsed
    ms_per_step = elapsed / K * 1e3

    # Roofline: each kernel's mean launch duration, HIP events (graph event
    # nodes on the launch stream) around L back-to-back launches of that
    # kernel alone, after the timed region. Event nodes between kernels would
    # add their own packet time to every launch.
    # Where a graph's time goes (outside the timed region): the timed graph
    # replayed three more times back to back (a busy GPU, as in the region),
    # HIP events on its stream around the third — the device time of a K-step
    # graph — against K x the settled per-step time of back-to-back launches
    # of the roofline's timing below
    graph_us = None
    if not eager and not stub:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        sync()
        run_steps(chunk, 0)
        run_steps(chunk, 0)
        e0.record()
        run_steps(chunk, 0)
        e1.record()
        sync()
        graph_us = e0.elapsed_time(e1) * 1e3

    roofline = None
    if not args.no_kernel_timing and not eager and not stub:
        roofline = kernel_roofline(env, cfg, actions, args, N, B, EL, roll, buf)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not stub:
        cpu = cpu_baseline(cfg, args.cpu_seconds, args.cpu_cores or host_cores())

    if rank == 0:
        P = W + A
        gb = world * B
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "agent-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("SELFTEST STUB (CPU stand-in env, not a measurement)" if stub else
                     "synthetic: Philox4x32-10 layouts, uniform random discrete actions pre-generated on device"),
            "config": {"workload": (f"cooperative_navigation {N} agents x {B} envs per GPU "
                                    f"({N} goals, {cfg.n_obstacles} obstacles; {cfg_name})") if not cfg.ragged
                       else f"{cfg.scenario} up to {N} agents x {B} envs per GPU ({cfg_name})",
                       "scenario": cfg.scenario, "n_agents": N, "n_envs_per_gpu": B, "global_envs": gb,
                       "agents_per_step": agents,
                       "episode_length": EL, "mean_edges_per_env": round(total_edges / B, 2),
                       "parallelism": f"env-sharded x{world} (no data-path collective)",
                       "launch": (f"GpuGraphVecEnv(output='numpy', graph='{(args.vec_env or '-').split('-')[1]}')"
                                  ".step(host int32 actions) per step: obs, agent_id, node_obs, adj as host arrays "
                                  "(per-agent axes as broadcast views of one host copy per table), rewards, costs, "
                                  "dones, LazyInfos" if args.vec_env else
                                  f"closed loop, one torch.cuda graph per {args.policy_graph_steps} step(s): greedy on-device policy(obs) "
                                  f"({'continuous sign(goal - pos), one kernel' if args.policy_act == 'cont' else 'discrete, three kernels'}) + "
                                  "GpuGraphVecEnv(output='torch', graph='coo').step (the one-launch step, device-side hand-off "
                                  "epoch)"
                                  if pgraph is not None else
                                  "closed loop: GpuGraphVecEnv(output='torch', graph='coo').step(policy(obs)) "
                                  "per step, greedy on-device policy" if venv is not None else
                                  "eager" if args.eager else ("rollout buffer (GraphRolloutBuffer.capture): "
                                  f"one launch per {EL}-step episode, step k's outputs into slot k+1 "
                                  "(node features, rewards, costs, done, CSR edges of every step at distinct "
                                  "addresses)" if buf is not None else "") + (f"hip-graphs of {chunk} steps" + (
                           (": all steps of a graph and their edges in one fused rollout launch (state on chip; "
                            + ("each env packs its edges a few steps behind its own step through a slab, "
                               "per-wave CSR prefix granules)" if cfg.ragged else "in-launch CSR look-back)"))
                           if roll else ", lagged emission (one launch per step)" if ((seg_cfg or cfg.ragged)
                                                                                     and not args.unfused)
                           else ", step + emit launch per step")))},
            "timed_region": {"untimed_steps_before": P + settle_steps, "align_steps": A,
                             "settle_steps": settle_steps,
                             "episode_boundaries": boundaries_in(P, K, EL),
                             "rank_ms_per_step_max": round(max(times) / K * 1e3, 5),
                             "rank_ms_per_step_min": round(min(times) / K * 1e3, 5),
                             **graph_breakdown(graph_us, roofline, chunk, n_chunks + (1 if rem else 0),
                                               elapsed, roll, buf is not None)},
            "episode_metrics": {"envs": gb, "finished_episodes": int(episodes),
                                "mean_last_episode_reward": round(ep_rew / gb, 4),
                                "mean_last_episode_cost": round(ep_cost / gb, 4),
                                "reduce": "all_reduce(SUM) over ranks" if pg else "single rank"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if lsa1 is not None:   # rank 0's polygon/line envs over the timed region
            hits, solved = lsa1[0] - lsa0[0], lsa1[1] - lsa0[1]
            line["assignment"] = {"warm_start_certified": hits, "assignments_solved": solved,
                                  "hit_rate": round(hits / solved, 6) if solved else None,
                                  "scope": "rank 0, timed region; the rest are solved cold"}
        print(json.dumps(line), flush=True)
    env.close()
    if pg:
        dist.destroy_process_group()
    return 0


def graph_breakdown(graph_us, roofline, chunk, n_graphs, elapsed, roll, buffer):
    """Split of the timed region per graph (rank 0): `graph_device_us` = HIP
    events around the third of three back-to-back replays of the timed graph
    right after the region (device time of a `chunk`-step graph); `settled_us` = chunk x the settled
    per-step time of back-to-back launches (the roofline's timing); `fill_us`
    = their difference, the graph's start and drain beyond its steps;
    `host_us` = wall time per graph in the region beyond the device time
    (launch call, synchronisation)."""
    if graph_us is None:
        return {}
    out = {"graph_steps": chunk, "graph_device_us": round(graph_us, 2),
           "host_us": round(elapsed / n_graphs * 1e6 - graph_us, 2)}
    step_us = (roofline or {}).get("mean_launch_us")
    if roll and step_us and not buffer:
        out["settled_us"] = round(chunk * step_us, 2)
        out["fill_us"] = round(graph_us - chunk * step_us, 2)
    return out


def counter_bound(pmc, ms, hbm_frac):
    """The roofline's counter-based figures, each a share of a
    measured ceiling, so none exceeds 1 by more than measurement noise:
    hbm_frac_physical = PMC HBM bytes / kernel time / 8 TB/s (what the kernel
    moves, against `frac`, which prices the contract's algorithmic bytes);
    valu_frac = VALU instructions / (SIMDs x launch cycles x VALU_PEAK);
    salu_frac = SALU instructions / (CUs x launch cycles x SALU_PEAK);
    wave_issue_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (the share of its
    resident time a wave spends issuing; the rest waits on memory / LDS /
    barriers or on a busy pipe). bound: the largest of the HBM, VALU and SALU
    shares when it reaches BOUND_AT ("hbm", or "issue" with the pipe named in
    binding_pipe), else "latency"."""
    out = dict(bound=None, traffic=None, hbm_frac_physical=None, valu_frac=None, salu_frac=None,
               wave_issue_frac=None, binding_pipe=None, counters=None)
    if not pmc:
        return out
    out["traffic"] = round(pmc["hbm_bytes_per_launch"])
    hbm_phys = pmc["hbm_bytes_per_launch"] / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9)
    out["hbm_frac_physical"] = round(hbm_phys, 4)
    cyc = pmc.get("grbm_gui_active_per_launch")
    shares = {"hbm": hbm_phys}
    if cyc:
        cyc = cyc / N_XCDS
        vf = pmc["valu_insts_per_launch"] / (N_SIMDS * cyc * VALU_PEAK)
        sf = pmc.get("salu_insts_per_launch", 0.0) / (N_CUS * cyc * SALU_PEAK)
        out.update(valu_frac=round(vf, 4), salu_frac=round(sf, 4))
        shares.update(valu=vf, salu=sf)
    if pmc.get("wave_quad_cycles_per_launch") and pmc.get("active_inst_any_quad_cycles_per_launch"):
        wc = pmc["wave_quad_cycles_per_launch"]
        out["wave_issue_frac"] = round(pmc["active_inst_any_quad_cycles_per_launch"] / wc, 4)
        waits = {k: round(pmc[f"{k}_quad_cycles_per_launch"] / wc, 4) for k in ("wait_any", "wait_inst_any")
                 if pmc.get(f"{k}_quad_cycles_per_launch")}
    else:
        waits = {}
    top = max(shares, key=shares.get)
    out["bound"] = ("hbm" if top == "hbm" else "issue") if shares[top] >= BOUND_AT else "latency"
    out["binding_pipe"] = top
    w = pmc.get("waves") or 1
    out["counters"] = dict(valu_insts_per_wave=round(pmc["valu_insts_per_launch"] / w, 1),
                           salu_insts_per_wave=round(pmc.get("salu_insts_per_launch", 0.0) / w, 1),
                           launch_cycles=round(cyc) if cyc else None, **waits,
                           ceilings=f"VALU {VALU_PEAK}/SIMD/cycle, SALU {SALU_PEAK}/CU/cycle "
                                    "(tools/probe_issue.hip), HBM 8 TB/s")
    return out


def kernel_roofline(env, cfg, actions, args, N, B, EL, roll=False, buf=None):
    import torch
    L = args.kernel_launches
    seg = (N + cfg.n_obstacles) <= 64 and not cfg.ragged
    lag = (seg or cfg.ragged) and not args.unfused and not roll   # segmented / ragged chains: lagged emission
    # the fused rollout: HIP events on the launch stream (torch's current
    # stream, where GpuBatchEnv launches) around R back-to-back launches of L
    # steps, time per step — the regime of the timed region and of rocprof's
    # average (one launch from idle measured ≈7% longer: the GPU ramps); the
    # chains: event nodes around the kernel in their graph
    if buf is not None:
        L = EL   # the buffer's episode graph (slot 0), timed as the rollout below
    if roll:
        if buf is None:
            env.capture(actions, L, slot=3, kernels="roll")
        rs = 0 if buf is not None else 3
        # settled like the timed region (--settle-ms of back-to-back launches
        # first: timed right after the region's host-side bookkeeping, the
        # first launches ran 5% slower while the GPU ramped back up)
        t_s = time.perf_counter()
        env.replay(rs)
        torch.cuda.synchronize()
        while (time.perf_counter() - t_s) * 1e3 < max(args.settle_ms, 5.0):
            env.replay(rs)
            torch.cuda.synchronize()
        R = 3
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(R):
            env.replay(rs)
        ev1.record()
        torch.cuda.synchronize()
        step_ms = ev0.elapsed_time(ev1) / R / L
    else:
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
        sb, eb, lb = ragged_kernel_bytes(env, EL, 4, edges_now)
        if lag:
            sb += lb
        names = ("gsm_step_ragged_kernel" + ("<lagged emission>" if lag else ""), "gsm_emit_ragged_kernel")
        if roll:
            sb = ragged_roll_step_bytes(env, EL, 4, edges_now)
            names = (f"gsm_roll_ragged_kernel (per step of a {L}-step launch)", names[1])
    elif roll:
        sb = roll_step_bytes(B, N, cfg.n_obstacles, EL, 4, edges_now, seg)
        eb = emit_kernel_bytes(B, N, cfg.n_obstacles, edges_now, seg)
        fam = "seg" if seg else "tile"
        names = (f"gsm_roll_{fam}_kernel{'<slots>' if buf is not None else ''} (per step of a {L}-step launch)",
                 f"gsm_emit_{fam}_kernel")
        if buf is not None:   # every step's node rows in full (all E rows of every slot)
            sb += B * (28 * (2 * N + cfg.n_obstacles - N)) * (1 - 1 / EL)
    else:
        sb = step_kernel_bytes(B, N, cfg.n_obstacles, EL, 4, seg, env.sizes.envs_per_block)
        if lag:
            sb += lag_extra_bytes(B, N, cfg.n_obstacles, edges_now, seg)
        eb = emit_kernel_bytes(B, N, cfg.n_obstacles, edges_now, seg)
        fam = "seg" if seg else "tile"
        names = (f"gsm_step_{fam}_kernel" + ("<lagged emission>" if lag else ""), f"gsm_emit_{fam}_kernel")
    # a launch that runs whole steps (a rollout step, a lagged step kernel:
    # physics, observation and the edges) is priced at SURVEY.md §8(d)'s
    # per-unit figure x the agents it steps — the contract's algorithmic bytes;
    # the kernel's own count of what it must move stays beside it
    kernel_bytes = sb
    bytes_model = "kernel count (bench.py step/emit/ragged_kernel_bytes)"
    if (roll or lag) and not cfg.ragged:
        sb = survey_bytes_per_agent_step(N, cfg.n_obstacles, 4, edges_now, B) * B * N
        bytes_model = "SURVEY.md §8(d) B_as per agent-step x agents per step"
    kern = {"step": dict(kernel=names[0], ms=step_ms, bytes=sb, gbs=sb / (step_ms * 1e-3) / 1e9),
            "emit": dict(kernel=names[1], ms=emit_ms, bytes=eb, gbs=eb / (emit_ms * 1e-3) / 1e9)}
    # a lagged chain / rollout runs the emit kernel once per graph, the step kernel every step
    dom = "step" if (lag or roll or step_ms >= emit_ms) else "emit"
    k = kern[dom]
    other = kern["emit" if dom == "step" else "step"]
    hbm_frac = k["gbs"] / HBM_PEAK_GBS
    pkey = f"{'roll' if (roll and dom == 'step') else 'lag' if (lag and dom == 'step') else dom}:{cfg.scenario}:N{N}:B{B}"
    if buf is not None and dom == "step":
        pkey = "rollbuf" + pkey[4:]
    pmc, note = pmc_entry(pkey)
    roofline = dict(kernel=k["kernel"], achieved=round(k["gbs"], 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(hbm_frac, 4), hbm_frac=round(hbm_frac, 4))
    roofline.update(counter_bound(pmc, k["ms"], hbm_frac))
    roofline.update(pmc=dict(key=pkey, status=note, source=pmc.get("source") if pmc else None),
                    algorithmic_bytes_per_launch=int(k["bytes"]),
                    bytes_model=bytes_model if dom == "step" else "kernel count",
                    kernel_bytes_per_launch=int(kernel_bytes) if dom == "step" else int(k["bytes"]),
                    # the same kernel priced at its own count of what it must
                    # move (a fused rollout keeps the state on chip: below the
                    # contract's §8(d) bytes), beside the contract's frac
                    kernel_bytes_frac=round((kernel_bytes if dom == "step" else k["bytes"]) /
                                            (k["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    mean_launch_us=round(k["ms"] * 1e3, 3),
                    timing=(f"HIP events around 3 back-to-back fused rollout launches of {L} steps (time per step)" if roll
                            else f"HIP events around {L} back-to-back graph launches of the kernel"),
                    other_kernel=dict(kernel=other["kernel"], achieved=round(other["gbs"], 1),
                                      algorithmic_bytes_per_launch=int(other["bytes"]),
                                      mean_launch_us=round(other["ms"] * 1e3, 3)))
    log(f"kernels: {json.dumps(kern)}")
    return roofline


if __name__ == "__main__":
    sys.exit(main())
