"""Multi-rank logic on CPU (gloo, world_size 2): env sharding by global env id
and the per-episode metric all-reduce (the only collective; RCCL on GPU)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsmarl_amd import EnvConfig
        from gsmarl_amd.distributed import all_reduce_metrics, max_over_ranks, shard_config
        from oracle import batch_ref as br
        cfg = shard_config(EnvConfig(n_agents=4, n_envs=3, seed=21), rank, world)
        # each rank's shard, computed by the oracle, equals the slice of the global batch
        ocfg = br.make_cfg(n_agents=4, n_envs=3, env_base=cfg.env_base, seed=21)
        local = br.new_state(ocfg, seed=21)["pos"]
        vec = torch.tensor([float(local.sum()), 1.0, float(rank)], dtype=torch.float64)
        all_reduce_metrics(vec)
        m = max_over_ranks(rank + 0.5)
        q.put((rank, cfg.env_base, cfg.n_envs, local, vec.numpy(), m))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_metric_allreduce():
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "gs-marl_amd")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    world = 2
    os.environ["PYTHONPATH"] = os.pathsep.join([str(root), str(root / "gs-marl_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    from oracle import batch_ref as br
    glob = br.new_state(br.make_cfg(n_agents=4, n_envs=6, seed=21), seed=21)["pos"]
    total = 0.0
    for rank, base, n, local, vec, m in res:
        assert base == rank * 3 and n == 3
        assert np.array_equal(local, glob[base:base + n])   # independent of the world size
        total += float(local.sum())
        assert m == pytest.approx(1.5)
    for *_, vec, _m in res:
        assert vec[0] == pytest.approx(total) and vec[1] == 2 and vec[2] == 1


def test_shard_config_strong_and_weak():
    from gsmarl_amd import EnvConfig
    from gsmarl_amd.distributed import shard_config
    c = EnvConfig(n_agents=24, n_envs=8192)
    assert [shard_config(c, r, 8).env_base for r in range(8)] == [r * 8192 for r in range(8)]
    s = shard_config(c, 3, 8, envs_per_rank=65536 // 8)
    assert s.n_envs == 8192 and s.env_base == 3 * 8192
    with pytest.raises(ValueError):
        shard_config(c, 8, 8)
