"""bench.py's multi-GPU rank body on one MI355X over RCCL: `--force-pg` joins
a one-rank "nccl" process group (RCCL) on cuda:0, so every collective the
driver's N-GPU run issues — the settle barrier, the MAX all-reduce of the
settle count, the barriers around the timed region, the all_gather of the
ranks' times and the SUM all-reduces of the episode metrics after it — runs
on hardware (BASELINE.json configs[4]). The
multi-rank logic itself is covered with gloo on CPU
(tests/test_bench_launcher.py)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_bench_rank_body_over_rccl_one_rank():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "1", "--steps", "20", "--warmup", "5",
                        "--no-cpu-baseline", "--settle-ms", "20", "--force-pg"],
                       capture_output=True, text=True, timeout=100, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["value"] > 0
    assert d["config"]["global_envs"] == 8192 and d["config"]["agents_per_step"] == 8192 * 24
    em = d["episode_metrics"]
    assert em["reduce"].startswith("all_reduce")
    # the timed region holds one auto-reset: every env finished at least one episode
    assert em["finished_episodes"] >= 8192
    tr = d["timed_region"]
    assert tr["episode_boundaries"] == 1
    assert tr["rank_ms_per_step_max"] == tr["rank_ms_per_step_min"] > 0
    # the region holds no collective but its barriers: its host time beyond
    # the 20-step graph stays within a barrier's (first launches of a metric
    # snapshot inside the region once put 42 ms there)
    assert tr["host_us"] < 200.0, tr
