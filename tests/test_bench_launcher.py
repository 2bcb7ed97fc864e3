"""bench.py's multi-rank launcher and rank body on CPU (gloo), with the GPU
env replaced by tests/bench_stub_env.py (`--selftest-env`): `--gpus N`
without torchrun spawns N ranks itself, never falls back to fewer, and rank 0
prints one line carrying the all-reduced episode metrics (BASELINE.json
configs[4])."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([str(ROOT / "tests"), str(ROOT / "gs-marl_amd"), str(ROOT),
                                         env.get("PYTHONPATH", "")])
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


def test_align_puts_an_episode_boundary_in_the_timed_region():
    sys.path.insert(0, str(ROOT))
    import bench
    EL = 100
    for W in (0, 1, 5, 50, 99, 100, 250):
        for K in (1, 2, 3, 10, 20, 99, 100, 101, 300):
            P = W + bench.align_steps(W, K, EL)
            assert bench.boundaries_in(P, K, EL) >= 1, (W, K)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gpus_n_spawns_n_ranks_and_reduces_metrics(world):
    B = 16
    # (world 1: --force-pg joins a one-rank group, so the collectives still run)
    r = _run(["--gpus", str(world), "--config", "c2", "--n-envs", str(B), "--steps", "20", "--warmup", "5",
              "--selftest-env", "bench_stub_env"] + (["--force-pg"] if world == 1 else []))
    assert r.returncode == 0, r.stderr[-2000:]
    # gloo logs its connection lines on stdout; the bench prints one JSON line (rank 0 only)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 20 and d["warmup"] == 5
    assert d["config"]["global_envs"] == world * B
    assert d["config"]["agents_per_step"] == world * B * 3
    assert d["data"].startswith("SELFTEST STUB")
    tr = d["timed_region"]
    assert tr["episode_boundaries"] == 1 and tr["untimed_steps_before"] == 90
    assert tr["rank_ms_per_step_max"] >= tr["rank_ms_per_step_min"] > 0
    em = d["episode_metrics"]
    # every env of every rank finished exactly one episode; rewards identify the global env ids
    gb = world * B
    assert em["finished_episodes"] == gb
    assert em["mean_last_episode_reward"] == pytest.approx(-sum(range(1, gb + 1)) / gb, abs=1e-4)
    assert em["reduce"].startswith("all_reduce")


def test_gpus_n_without_gpus_fails_instead_of_falling_back():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "GPU(s) visible" in r.stderr


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--steps", "2", "--selftest-env", "bench_stub_env"], {"WORLD_SIZE": "1"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr and r.stdout.strip() == ""


def test_multi_chunk_region_reduces_metrics_after_it():
    """A 250-step region (chunks of 100, 100 and a 50-step remainder): the
    line's metrics are the all-reduced totals after the region."""
    B, world = 16, 2
    r = _run(["--gpus", str(world), "--config", "c2", "--n-envs", str(B), "--steps", "250", "--warmup", "5",
              "--selftest-env", "bench_stub_env"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["steps"] == 250 and d["timed_region"]["episode_boundaries"] == 3
    em = d["episode_metrics"]
    assert em["reduce"].startswith("all_reduce") and em["finished_episodes"] == 3 * world * B
