"""BASELINE configs[4] (C5: 24 agents x 65536 envs over 8 MI355X) on one GPU.

C5 shards the envs by global id: rank r steps envs [r * 8192, (r + 1) * 8192)
with ``env_base = r * 8192`` (gsmarl_amd.distributed.shard_config), and every
Philox layout is keyed by the global env id, so a rank's shard must be, bit
for bit, its slice of the one 65536-env batch — the only cross-GPU step is the
RCCL reduce of episode metrics. Here ranks
0, 3 and 7 are stepped on one GPU through the fused rollout (every step into a
rollout buffer's slots, and the headline in-place rollout kernel) and compared
with one 65536-env batch stepped eagerly from the same actions over a 100-step
episode (the auto-reset re-lays every env out in the last step): node
features, rewards, costs, done, edge counts, the CSR offsets and edges
re-based to the shard's node ids, and the final state. Rank 7's shard is also
checked against the CPU oracle on a sample of envs (reset layouts bit-exact,
positions / velocities of every step within the 1e-6 bar, edges exact)."""
import numpy as np
import pytest
import torch

from oracle import batch_ref as br
from parity_tol import check_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N, B_ALL, B_RANK, T, SEED = 24, 65536, 8192, 100, 77
RANKS = (0, 3, 7)
STATE = ("pos", "vel", "step_count", "episode", "ep_acc", "ep_last")


def _env(n_envs, env_base=0):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    cfg = EnvConfig(n_agents=N, n_envs=n_envs, env_base=env_base, seed=SEED, episode_length=T)
    return GpuBatchEnv(cfg, DEV), cfg


def _sample_oracle(buf, acts, r, cfg):
    """Rank r's shard vs the oracle on a sample of its envs, every step."""
    sel = np.array([0, 1, 2047, 4096, 8190, 8191])
    E = buf.E
    ocfg = br.make_cfg(n_agents=N, n_envs=len(sel), episode_length=T, seed=SEED)
    nf = buf.node_feat[:, sel].cpu().numpy()            # [T+1, S, E, 7]
    a = acts[:, sel].cpu().numpy()
    gids = r * B_RANK + sel
    # slot 0: the reset layout of episode 0, slot T: episode 1's (the auto-reset)
    for slot, ep in ((0, 0), (T, 1)):
        want = br.layout(ocfg, gids, np.full(len(sel), ep), seed=SEED)
        assert np.array_equal(nf[slot, :, :, 2:4], want), ("layout", slot)
    for t in range(T - 1):   # (step T - 1 ends the episode: slot T holds the new layout)
        pos, vel = nf[t, :, :, 2:4].astype(np.float64), nf[t, :, :N, 0:2].astype(np.float64)
        p64, v64 = br.physics(ocfg, pos, vel, a[t], 1, np.float64)
        check_state(nf[t + 1, :, :, 2:4], p64, f"pos r{r} t{t}")
        check_state(nf[t + 1, :, :N, 0:2], v64, f"vel r{r} t{t}")
    # the last in-episode step's edges, exact (fp32-mode oracle on the kernel's positions)
    t = T - 1
    ptr, ei, _ = br.edges(ocfg, nf[t, :, :, 2:4], np.float32)
    g_ptr = buf.edge_ptr[t].cpu().numpy()
    g_ei = buf.edge_index[t].cpu().numpy()
    for j, b in enumerate(sel):
        got = g_ei[:, g_ptr[b]:g_ptr[b + 1]] - b * E
        exp = ei[:, ptr[j]:ptr[j + 1]] - j * E
        assert np.array_equal(got, exp), (r, b)


def test_c5_shards_equal_slices_of_one_batch():
    from gsmarl_amd import GraphRolloutBuffer
    gen = torch.Generator(device=DEV)
    gen.manual_seed(SEED)
    acts = torch.randint(0, 5, (T, B_ALL, N), dtype=torch.int32, device=DEV, generator=gen)
    shards = {}
    for r in RANKS:
        env, cfg = _env(B_RANK, env_base=r * B_RANK)
        sl = acts[:, r * B_RANK:(r + 1) * B_RANK].contiguous()
        buf = GraphRolloutBuffer(env, episode_length=T)
        buf.reset(seed=SEED)
        buf.capture(sl)
        assert env.graph_is_rollout(0), "the shard's episode runs as one fused rollout launch"
        buf.replay()
        buf.validate()
        assert not bool(buf.overflowed())
        # the headline form: the same episode in one in-place rollout launch
        env.reset(seed=SEED)
        env.capture(sl, T, slot=1, kernels="roll")
        env.replay(1)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        final = {k: env.t[k].clone() for k in STATE}
        shards[r] = (env, cfg, buf, sl, final)
        if r == 7:
            _sample_oracle(buf, sl, r, cfg)

    big, bcfg = _env(B_ALL)
    big.reset(seed=SEED, sync_edges=False)
    E = big.E
    for t in range(T):
        big.step(acts[t], sync_edges=False)
        ptr = big.t["edge_ptr"]
        for r, (env, cfg, buf, sl, final) in shards.items():
            r0, r1 = r * B_RANK, (r + 1) * B_RANK
            s = t + 1
            for k in ("node_feat", "reward", "cost", "done", "edge_count"):
                assert torch.equal(big.t[k][r0:r1], getattr(buf, k)[s]), (r, t, k)
            p0, p1 = int(ptr[r0]), int(ptr[r1])
            assert torch.equal(ptr[r0:r1 + 1] - p0, buf.edge_ptr[s]), (r, t, "edge_ptr")
            n = p1 - p0
            assert torch.equal(big.t["edge_index"][:, p0:p1] - r0 * E, buf.edge_index[s][:, :n]), (r, t, "edges")
            assert torch.equal(big.t["edge_attr"][p0:p1], buf.edge_attr[s][:n]), (r, t, "edge_attr")
    torch.cuda.synchronize()
    assert int(big.t["done"].sum()) == B_ALL and int(big.t["episode"].min()) == 1   # every env auto-reset
    for r, (env, cfg, buf, sl, final) in shards.items():
        r0, r1 = r * B_RANK, (r + 1) * B_RANK
        for k in STATE:
            assert torch.equal(big.t[k][r0:r1], final[k]), (r, k)
        # the in-place rollout's last-step outputs are the buffer's last slot
        for k in ("node_feat", "reward", "cost", "done", "edge_count", "edge_ptr"):
            assert torch.equal(env.t[k], getattr(buf, k)[T]), (r, k)
        n = int(env.t["edge_ptr"][-1])
        assert torch.equal(env.t["edge_index"][:, :n], buf.edge_index[T][:, :n]), r
        env.close()
    big.close()


def test_ragged_shards_equal_slices_of_one_batch():
    """The ragged (C4-style mixed) path sharded the same way: a scenario of
    global id mod 3 and an N_env drawn from the global id, so two 8192-env
    shards (env_base 0 and 8192) stepped through the fused ragged rollout
    into rollout-buffer slots equal, step for step, their slices of one
    16384-env batch stepped eagerly — node features, rewards, costs, done,
    assignments, CSR edges re-based, and the final state with the
    assignment warm-start duals — over 30 steps with an auto-reset at 20."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
    Nm, BA, BR, TT, EL = 24, 16384, 8192, 30, 20
    kw = dict(scenario="mixed", n_agents=Nm, n_agents_min=3, seed=SEED, episode_length=EL)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(SEED + 1)
    acts = torch.randint(0, 5, (TT, BA, Nm), dtype=torch.int32, device=DEV, generator=gen)
    shards = {}
    for r in (0, 1):
        env = GpuBatchEnv(EnvConfig(n_envs=BR, env_base=r * BR, **kw), DEV)
        buf = GraphRolloutBuffer(env, episode_length=TT)
        buf.reset(seed=SEED)
        buf.capture(acts[:, r * BR:(r + 1) * BR].contiguous())
        assert env.graph_is_rollout(0)
        buf.replay()
        buf.validate()
        assert not bool(buf.overflowed())
        torch.cuda.synchronize()
        shards[r] = (env, buf)
    big = GpuBatchEnv(EnvConfig(n_envs=BA, **kw), DEV)
    big.reset(seed=SEED, sync_edges=False)
    E = big.E
    for t in range(TT):
        big.step(acts[t], sync_edges=False)
        ptr = big.t["edge_ptr"]
        for r, (env, buf) in shards.items():
            r0, r1, s = r * BR, (r + 1) * BR, t + 1
            for k in ("node_feat", "reward", "cost", "done", "edge_count", "assign"):
                assert torch.equal(big.t[k][r0:r1], getattr(buf, k)[s]), (r, t, k)
            p0, p1 = int(ptr[r0]), int(ptr[r1])
            assert torch.equal(ptr[r0:r1 + 1] - p0, buf.edge_ptr[s]), (r, t, "edge_ptr")
            n = p1 - p0
            assert torch.equal(big.t["edge_index"][:, p0:p1] - r0 * E, buf.edge_index[s][:, :n]), (r, t, "edges")
            assert torch.equal(big.t["edge_attr"][p0:p1], buf.edge_attr[s][:n]), (r, t, "edge_attr")
    torch.cuda.synchronize()
    for r, (env, buf) in shards.items():
        r0, r1 = r * BR, (r + 1) * BR
        for k in STATE + ("env_shape", "lsa_v", "lsa_col"):
            assert torch.equal(big.t[k][r0:r1], env.t[k]), (r, k)
        env.close()
    big.close()
