"""HIP step path vs the CPU oracle, through the C ABI (libgsm.so).

Tolerances (north_star): positions/velocities within 1e-6 (absolute) of the
fp64 oracle stepped from the *identical* fp32 state (tests/parity_tol.py: a
4-ulp term only where |x| >= 8, where one fp32 ulp is ~1e-6; the largest error
seen per test is printed at the end of the run); collision-cost counts, edge_ptr and
edge_index bit-exact vs the fp32-mode oracle evaluated on the kernel's own
fp32 positions; node features bit-exact; rewards and edge distances within
2 fp32 ulp.
"""
import numpy as np
import pytest
import torch

from oracle import batch_ref as br
from parity_tol import check_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cfgs(**kw):
    from gsmarl_amd import EnvConfig
    cfg = EnvConfig(**kw)
    ocfg = br.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in br.DEFAULTS})
    return cfg, ocfg


def _env(**kw):
    from gsmarl_amd import GpuBatchEnv
    cfg, ocfg = _cfgs(**kw)
    return GpuBatchEnv(cfg, DEV), ocfg


def _np(t):
    return t.detach().cpu().numpy()


def assert_state_close(got, ref, what):
    check_state(got, ref, what)


def check_outputs(env, ocfg, out):
    """Integer outputs bit-exact, float outputs within tolerance, from the
    kernel's own post-step fp32 state."""
    pos, vel = _np(env.t["pos"]), _np(env.t["vel"])
    ptr, ei, attr = br.edges(ocfg, pos, np.float32)
    assert np.array_equal(_np(out["edge_ptr"]), ptr), "edge_ptr"
    assert np.array_equal(_np(out["edge_index"]), ei), "edge_index"
    assert np.allclose(_np(out["edge_attr"]), attr, rtol=2.5e-7, atol=0), "edge_attr"
    nf = br.node_features(ocfg, pos, vel, np.float32)
    assert np.array_equal(_np(out["node_feat"]), nf), "node_feat"
    assert np.array_equal(_np(out["obs"]), nf[:, : ocfg.n_agents, :6]), "obs view"
    assert np.array_equal(_np(env.t["edge_count"]), np.diff(ptr).astype(np.int32)), "edge_count"


def check_cost_reward(env, ocfg, out):
    pos = _np(env.t["pos"])
    r, c = br.reward_cost(ocfg, pos, np.float32)
    assert np.array_equal(_np(out["cost"]), c), "cost"
    r64, _ = br.reward_cost(ocfg, pos.astype(np.float64), np.float64)
    assert np.allclose(_np(out["reward"]), r64, rtol=3e-7, atol=1e-6), "reward"


# ------------------------------------------------------------------ reset
@pytest.mark.parametrize("N,B", [(3, 1), (3, 4096), (24, 512), (96, 64), (1, 8), (65, 4)])
def test_reset_layout_bit_exact(N, B):
    env, ocfg = _env(n_agents=N, n_envs=B, seed=11)
    out = env.reset(seed=11)
    torch.cuda.synchronize()
    ref = br.new_state(ocfg, seed=11, dtype=np.float32)
    assert np.array_equal(_np(env.t["pos"]), ref["pos"])
    assert np.all(_np(env.t["episode"]) == 0) and np.all(_np(env.t["step_count"]) == 0)
    check_outputs(env, ocfg, out)
    check_cost_reward(env, ocfg, out)


def test_reset_mask_and_reseed():
    env, ocfg = _env(n_agents=5, n_envs=6, seed=1)
    env.reset(seed=1)
    p0 = _np(env.t["pos"]).copy()
    mask = torch.tensor([0, 1, 0, 0, 1, 0], dtype=torch.uint8)
    out = env.reset(env_mask=mask)
    p1 = _np(env.t["pos"])
    ep = _np(env.t["episode"])
    assert ep.tolist() == [0, 1, 0, 0, 1, 0]
    assert np.array_equal(p1[[0, 2, 3, 5]], p0[[0, 2, 3, 5]])
    lay = br.layout(ocfg, [1, 4], [1, 1], 1)
    assert np.array_equal(p1[[1, 4]], lay)
    check_outputs(env, ocfg, out)
    env.reset(seed=1)
    assert np.array_equal(_np(env.t["pos"]), p0)


# ------------------------------------------------------------------ physics
def _inject_random(env, ocfg, L, seed, vel_scale=1.0):
    rng = np.random.default_rng(seed)
    B, N, E = env.B, env.N, env.E
    pos = rng.uniform(-L, L, size=(B, E, 2)).astype(np.float32)
    vel = (vel_scale * rng.normal(size=(B, N, 2))).astype(np.float32)
    env.set_state(dict(pos=torch.from_numpy(pos), vel=torch.from_numpy(vel)))
    torch.cuda.synchronize()
    return pos, vel


@pytest.mark.parametrize("N,No,B,L", [(3, 3, 64, 0.35), (24, 24, 256, 1.2), (24, 24, 256, 2.83), (5, 2, 37, 0.5), (32, 32, 9, 1.6), (24, 24, 8, 0.3), (8, 8, 16, 0.2),
                                      (96, 96, 16, 3.0), (64, 0, 8, 1.0), (65, 7, 8, 1.5), (1, 0, 4, 1.0),
                                      (600, 10, 2, 8.0), (40, 40, 8, 0.9), (3, 3, 4096, 1.0),
                                      (3, 3, 4096, 0.3), (24, 24, 8192, 2.83)])
def test_one_step_physics_parity(N, No, B, L):
    env, ocfg = _env(n_agents=N, n_obstacles=No, n_envs=B, episode_length=1000)
    if (N, No, B) == (3, 3, 4096):   # C2: the specialised <3,3> kernels, 4 envs per wave
        assert env.sizes.envs_per_block == 16
    env.reset(seed=0)
    pos, vel = _inject_random(env, ocfg, L, seed=N + B)
    rng = np.random.default_rng(5)
    for fmt in ("index", "onehot", "cont"):
        env.set_state(dict(pos=torch.from_numpy(pos), vel=torch.from_numpy(vel)))
        a = rng.integers(0, 5, size=(B, N))
        if fmt == "index":
            act, f, an = torch.from_numpy(a.astype(np.int32)).to(DEV), 1, a
        elif fmt == "onehot":
            an = np.eye(5, dtype=np.float32)[a]
            act, f = torch.from_numpy(an).to(DEV), 0
        else:
            an = rng.uniform(-1, 1, size=(B, N, 2)).astype(np.float32)
            act, f = torch.from_numpy(an).to(DEV), 2
        out = env.step(act)
        torch.cuda.synchronize()
        p64, v64 = br.physics(ocfg, pos.astype(np.float64), vel.astype(np.float64), an, f, np.float64)
        assert_state_close(_np(env.t["pos"]), p64, f"pos ({fmt})")
        assert_state_close(_np(env.t["vel"]), v64, f"vel ({fmt})")
        check_outputs(env, ocfg, out)
        check_cost_reward(env, ocfg, out)


def test_onehot_and_index_bitwise_identical():
    env, ocfg = _env(n_agents=24, n_envs=128)
    env.reset(seed=4)
    s0 = env.get_state()
    a = torch.randint(0, 5, (128, 24), dtype=torch.int32, device=DEV)
    o1 = {k: v.clone() for k, v in env.step(a).items()}
    p1 = env.t["pos"].clone()
    env.set_state(s0)
    o2 = env.step(torch.nn.functional.one_hot(a.long(), 5).float())
    assert torch.equal(p1, env.t["pos"])
    for k in ("reward", "cost", "node_feat", "edge_index", "edge_attr", "edge_ptr"):
        assert torch.equal(o1[k], o2[k]), k


def test_max_speed_clamp_parity():
    env, ocfg = _env(n_agents=8, n_envs=32, max_speed=0.3)
    env.reset(seed=2)
    pos, vel = _inject_random(env, ocfg, 0.6, seed=3, vel_scale=2.0)
    a = np.random.default_rng(1).integers(0, 5, size=(32, 8))
    env.step(torch.from_numpy(a.astype(np.int32)).to(DEV))
    p64, v64 = br.physics(ocfg, pos.astype(np.float64), vel.astype(np.float64), a, 1, np.float64)
    assert_state_close(_np(env.t["vel"]), v64, "vel")
    assert_state_close(_np(env.t["pos"]), p64, "pos")
    assert np.all(np.linalg.norm(_np(env.t["vel"]), axis=-1) <= 0.3 + 1e-6)


def test_boundary_predicates_exact():
    """Pairs exactly at the collision distance and at the sensing radius."""
    env, ocfg = _env(n_agents=2, n_obstacles=1, n_envs=1)
    env.reset(seed=0)
    dmin = np.float32(0.05) + np.float32(0.05)
    pos = np.array([[[0.0, 0.0], [dmin, 0.0], [2.0, 2.0], [-2.0, 2.0], [0.0, 0.5]]], np.float32)
    out = env.set_state(dict(pos=torch.from_numpy(pos), vel=torch.zeros(1, 2, 2)))
    torch.cuda.synchronize()
    assert _np(out["cost"]).tolist() == [[0.0, 0.0]]          # d2 == dmin2: strict
    ei = _np(out["edge_index"])
    assert (0, 4) in set(zip(ei[0].tolist(), ei[1].tolist()))  # d2 == R2: inclusive
    check_outputs(env, ocfg, out)
    pos[0, 1, 0] = np.nextafter(dmin, np.float32(0))
    out = env.set_state(dict(pos=torch.from_numpy(pos)))
    assert _np(out["cost"]).tolist() == [[1.0, 1.0]]
    # coincident agents: guarded force, counted collision, no radius edge
    pos[0, 1] = pos[0, 0]
    env.set_state(dict(pos=torch.from_numpy(pos), vel=torch.zeros(1, 2, 2)))
    out = env.step(torch.zeros(1, 2, dtype=torch.int32, device=DEV))
    assert np.all(np.isfinite(_np(env.t["pos"])))
    check_outputs(env, ocfg, out)


def test_coincident_pairs_one_env_per_wave():
    """24 agents (one env per wave, the headline sweep): a coincident
    agent-agent and agent-obstacle pair count as collisions, give no radius
    edge and no contact force, through set_state (full sweep) and a step."""
    N, B = 24, 4
    env, ocfg = _env(n_agents=N, n_envs=B)
    env.reset(seed=0)
    E = 3 * N
    rng = np.random.default_rng(5)
    gx, gy = np.meshgrid(np.arange(9), np.arange(8))
    grid = (np.stack([gx.ravel(), gy.ravel()], -1)[:E] * 0.62 - 2.5).astype(np.float32)
    pos = np.stack([grid + rng.uniform(-0.05, 0.05, grid.shape).astype(np.float32) for _ in range(B)])
    pos[1, 7] = pos[1, 3]                # agent-agent
    pos[1, 5] = pos[1, 2 * N + 2]        # agent-obstacle
    pos[2, 0] = pos[2, 2 * N]            # agent-obstacle, obstacle 0
    out = env.set_state(dict(pos=torch.from_numpy(pos), vel=torch.zeros(B, N, 2)))
    torch.cuda.synchronize()
    check_outputs(env, ocfg, out)
    check_cost_reward(env, ocfg, out)
    assert _np(out["cost"])[1, [3, 7, 5]].tolist() == [1.0, 1.0, 1.0]
    for _ in range(2):
        out = env.step(torch.zeros(B, N, dtype=torch.int32, device=DEV))
        torch.cuda.synchronize()
        assert np.all(np.isfinite(_np(env.t["pos"])))
        check_outputs(env, ocfg, out)
        check_cost_reward(env, ocfg, out)
    p = _np(env.t["pos"])
    assert np.array_equal(p[1, 7], p[1, 3]) and np.array_equal(p[1, 5], p[1, 2 * N + 2])
    assert _np(out["cost"])[2, 0] == 1.0


# ------------------------------------------------------------- episodes
@pytest.mark.parametrize("N,B", [(3, 1), (3, 256), (24, 64), (96, 16), (40, 8)])
def test_episode_rollout_stepwise(N, B):
    """A 2.5-episode rollout with auto-reset; each step is checked against the
    fp64 oracle started from the kernel's own pre-step state."""
    env, ocfg = _env(n_agents=N, n_envs=B, episode_length=20, seed=7)
    env.reset(seed=7)
    rng = np.random.default_rng(N)
    for t in range(50):
        st = {k: _np(v) for k, v in env.get_state().items()}
        ref_st = dict(pos=st["pos"].astype(np.float64), vel=st["vel"].astype(np.float64),
                      step=st["step_count"], episode=st["episode"],
                      ep_acc=st["ep_acc"].astype(np.float64), ep_last=st["ep_last"].astype(np.float64))
        a = rng.integers(0, 5, size=(B, N))
        out = env.step(torch.from_numpy(a.astype(np.int32)).to(DEV))
        torch.cuda.synchronize()
        nst, ob = br.step(ocfg, ref_st, a, 1, np.float64, seed=7)
        done = _np(out["done"]).astype(bool)
        assert np.array_equal(done, ob["done"].astype(bool))
        assert np.array_equal(_np(env.t["step_count"]), nst["step"])
        assert np.array_equal(_np(env.t["episode"]), nst["episode"])
        assert_state_close(_np(env.t["pos"]), nst["pos"], f"pos t={t}")
        assert_state_close(_np(env.t["vel"]), nst["vel"], f"vel t={t}")
        # episode accounting from the kernel's own per-step outputs
        acc_exp = st["ep_acc"].astype(np.float64) + np.stack(
            [_np(out["reward"]).astype(np.float64).sum(-1), _np(out["cost"]).astype(np.float64).sum(-1)], -1)
        if done.any():    # re-laid-out envs are bit-exact
            lay = br.layout(ocfg, np.nonzero(done)[0], nst["episode"][done], 7)
            assert np.array_equal(_np(env.t["pos"])[done], lay)
            assert np.allclose(_np(env.t["ep_last"])[done], acc_exp[done], rtol=1e-5, atol=1e-4)
            acc_exp[done] = 0
        assert np.allclose(_np(env.t["ep_acc"]), acc_exp, rtol=1e-5, atol=1e-4)
        # cost exact (fp32 predicate) on the post-physics state of envs that did not reset
        keep = ~done
        if keep.any():
            _, c32 = br.reward_cost(ocfg, _np(env.t["pos"])[keep], np.float32)
            assert np.array_equal(_np(out["cost"])[keep], c32)
        check_outputs(env, ocfg, out)
        assert np.allclose(_np(out["reward"]), ob["reward"], rtol=3e-7, atol=2e-6)


def test_shared_reward():
    env, ocfg = _env(n_agents=6, n_envs=16, shared_reward=True)
    env.reset(seed=3)
    out = env.step(torch.zeros(16, 6, dtype=torch.int32, device=DEV))
    r64, _ = br.reward_cost(ocfg, _np(env.t["pos"]).astype(np.float64), np.float64)
    assert np.allclose(_np(out["reward"]), r64, rtol=1e-6, atol=1e-5)


# ------------------------------------------------------- graph & determinism
def test_graph_replay_equals_eager_and_deterministic():
    env, ocfg = _env(n_agents=24, n_envs=256, episode_length=30)
    T = 40
    acts = torch.randint(0, 5, (T, 256, 24), dtype=torch.int32, device=DEV)
    env.reset(seed=5)
    for t in range(T):
        env.step(acts[t], sync_edges=False)
    eager = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=5)
    env.capture(acts, T, timing=True)
    env.replay()
    torch.cuda.synchronize()
    for k in ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "edge_ptr",
              "edge_index", "edge_attr", "ep_acc", "ep_last"):
        assert torch.equal(eager[k], env.t[k]), k
    a, b, tot = env.graph_kernel_ms()
    assert a > 0 and b > 0 and tot >= T * (a + b) * 0.99
    env.reset(seed=5)
    env.replay()
    torch.cuda.synchronize()
    assert torch.equal(eager["edge_index"], env.t["edge_index"])
    assert torch.equal(eager["pos"], env.t["pos"])


@pytest.mark.parametrize("N,B,T", [(24, 256, 40), (24, 257, 7), (3, 4000, 1), (3, 123, 2), (5, 37, 9), (7, 64, 6),
                                   (70, 9, 3), (96, 17, 6), (3, 4096, 7), (3, 4100, 6)])
def test_lagged_chain_equals_eager(N, B, T):
    """Segmented graphs emit step j's edges from step j+1's kernel (lagged
    emission): the chain must leave every state and output buffer exactly as
    eager steps and as the two-kernel chain do, for odd and even chain
    lengths, partial workgroups and auto-resets (episode length 5). Tile
    shapes (M > 64) run the two-kernel chain under both names."""
    env, ocfg = _env(n_agents=N, n_envs=B, episode_length=5)
    if N == 3 and B >= 4096:   # C2's specialised <3,3> kernels (4 envs per wave)
        assert env.sizes.envs_per_block == 16
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    keys = ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "done", "edge_count",
            "edge_ptr", "ep_acc", "ep_last", "row_mask", "contact_mask")
    env.reset(seed=6)
    for t in range(T):
        env.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    eager = {k: v.clone() for k, v in env.t.items()}
    n = int(eager["edge_ptr"][-1])
    for kernels, slot in (("both", 0), ("unfused", 1)):
        env.reset(seed=6)
        env.capture(acts, T, slot=slot, kernels=kernels)
        env.replay(slot)
        torch.cuda.synchronize()
        for k in keys:
            assert torch.equal(eager[k], env.t[k]), (kernels, k)
        assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n]), kernels
        assert torch.equal(eager["edge_attr"][:n], env.t["edge_attr"][:n]), kernels
        # the bound edge-sum buffer holds the last step's sums: an emit-only
        # graph right after the chain re-emits the same edges
        env.t["edge_index"].zero_()
        env.capture(None, 1, slot=3, kernels="emit")
        env.replay(3)
        torch.cuda.synchronize()
        assert torch.equal(eager["edge_ptr"], env.t["edge_ptr"]), kernels
        assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n]), kernels
    env.close()


@pytest.mark.parametrize("N,B", [(24, 300), (5, 41)])
def test_lag_only_graph(N, B):
    """The lagged-kernel timing graph: physics like eager steps; its last
    emission is that of the step before the last."""
    env, ocfg = _env(n_agents=N, n_envs=B, episode_length=1000)
    T = 6
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=9)
    for t in range(T - 1):
        env.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    before_last = {k: env.t[k].clone() for k in ("edge_ptr", "edge_index", "edge_attr")}
    env.step(acts[T - 1], sync_edges=False)
    eager = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=9)
    env.capture(acts, T, slot=2, kernels="lag", time_ends=True)
    env.replay(2)
    torch.cuda.synchronize()
    for k in ("pos", "vel", "step_count", "node_feat", "reward", "cost", "edge_count"):
        assert torch.equal(eager[k], env.t[k]), k
    n = int(before_last["edge_ptr"][-1])
    assert torch.equal(before_last["edge_ptr"], env.t["edge_ptr"])
    assert torch.equal(before_last["edge_index"][:, :n], env.t["edge_index"][:, :n])
    assert torch.equal(before_last["edge_attr"][:n], env.t["edge_attr"][:n])
    s_ms, e_ms, tot = env.graph_kernel_ms(2)
    assert s_ms > 0 and e_ms == 0
    env.close()


def test_kernel_only_graphs():
    """Roofline timing graphs: a step-only graph advances the physics exactly
    like eager steps; an emit-only graph re-emits the same edges (idempotent)."""
    env, ocfg = _env(n_agents=24, n_envs=512, episode_length=1000)
    T = 12
    acts = torch.randint(0, 5, (T, 512, 24), dtype=torch.int32, device=DEV)
    env.reset(seed=8)
    for t in range(T):
        env.step(acts[t], sync_edges=False)
    eager = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=8)
    env.capture(acts, T, slot=3, kernels="step", time_ends=True)
    env.replay(3)
    torch.cuda.synchronize()
    for k in ("pos", "vel", "step_count", "reward", "cost", "node_feat", "edge_count"):
        assert torch.equal(eager[k], env.t[k]), k
    s_ms, e_ms, tot = env.graph_kernel_ms(3)
    assert s_ms > 0 and e_ms == 0 and abs(s_ms * T - tot) < 1e-6 * T + 1e-3
    env.capture(None, 5, slot=3, kernels="emit", time_ends=True)
    env.replay(3)
    torch.cuda.synchronize()
    n = int(eager["edge_ptr"][-1])   # beyond it: stale entries of earlier steps
    assert torch.equal(eager["edge_ptr"], env.t["edge_ptr"])
    assert torch.equal(eager["edge_index"][:, :n], env.t["edge_index"][:, :n])
    assert torch.equal(eager["edge_attr"][:n], env.t["edge_attr"][:n])
    assert env.graph_kernel_ms(3)[1] > 0


def test_c3_size_sample():
    """BASELINE C3 (96 agents x 1024 envs, tile path): three steps, then the
    oracle on a sample of envs from the kernel's own state."""
    env, ocfg = _env(n_agents=96, n_envs=1024, episode_length=1000)
    env.reset(seed=2)
    rng = np.random.default_rng(2)
    for _ in range(3):
        st = {k: _np(v) for k, v in env.get_state().items()}
        a = rng.integers(0, 5, size=(1024, 96))
        out = env.step(torch.from_numpy(a.astype(np.int32)).to(DEV))
        torch.cuda.synchronize()
    idx = np.array([0, 1, 511, 1022, 1023])
    p64, v64 = br.physics(ocfg, st["pos"][idx].astype(np.float64), st["vel"][idx].astype(np.float64),
                          a[idx], 1, np.float64)
    assert_state_close(_np(env.t["pos"])[idx], p64, "pos")
    assert_state_close(_np(env.t["vel"])[idx], v64, "vel")
    pos = _np(env.t["pos"])
    ptr, ei, attr = br.edges(ocfg, pos, np.float32)
    assert np.array_equal(_np(out["edge_ptr"]), ptr)
    assert np.array_equal(_np(out["edge_index"]), ei)
    _, c = br.reward_cost(ocfg, pos, np.float32)
    assert np.array_equal(_np(out["cost"]), c)


def test_headline_size_properties():
    """Full BASELINE headline config (24 agents x 8192 envs): size-independent
    properties of the graph output + oracle parity on a sample of envs."""
    env, ocfg = _env(n_agents=24, n_envs=8192)
    env.reset(seed=0)
    acts = torch.randint(0, 5, (8192, 24), dtype=torch.int32, device=DEV)
    for _ in range(3):
        out = env.step(acts)
    torch.cuda.synchronize()
    ptr = out["edge_ptr"]
    ei = out["edge_index"].long()
    E = env.E
    assert int(ptr[0]) == 0 and bool((ptr[1:] >= ptr[:-1]).all())
    cnt = (ptr[1:] - ptr[:-1])
    assert torch.equal(cnt.to(torch.int32), env.t["edge_count"])
    env_of_edge = torch.repeat_interleave(torch.arange(8192, device=DEV), cnt)
    assert torch.equal(ei[0] // E, env_of_edge) and torch.equal(ei[1] // E, env_of_edge)
    key = ei[0] * (E * 8192) + ei[1]
    assert bool((key[1:] > key[:-1]).all()), "row-major, strictly increasing"
    rev = ei[1] * (E * 8192) + ei[0]
    assert torch.equal(torch.sort(rev).values, key), "edge set symmetric"
    assert bool((out["edge_attr"] >= 0).all())
    # recount the radius predicate with torch (separate mul/add kernels, no FMA)
    pos = env.t["pos"]
    N = 24
    ao = torch.cat([pos[:, :N], pos[:, 2 * N:]], 1)
    dx = ao[:, :, None, 0] - ao[:, None, :, 0]
    dy = ao[:, :, None, 1] - ao[:, None, :, 1]
    d2 = dx * dx + dy * dy
    R2 = torch.tensor(np.float32(0.5) * np.float32(0.5), device=DEV)
    n_rad = ((d2 > 0) & (d2 <= R2)).sum((1, 2))
    assert torch.equal((n_rad + 2 * N).to(torch.int32), env.t["edge_count"])
    # exact oracle parity on a sample of envs
    sel = np.arange(0, 8192, 97)
    pos_np = _np(pos)[sel]
    p_, e_, a_ = br.edges(br.make_cfg(n_agents=24, n_envs=len(sel)), pos_np, np.float32)
    ptr_np, ei_np = _np(ptr), _np(out["edge_index"])
    for j, b in enumerate(sel):
        got = ei_np[:, ptr_np[b]:ptr_np[b + 1]] - b * E
        exp = e_[:, p_[j]:p_[j + 1]] - j * E
        assert np.array_equal(got, exp), b


def test_dropin_graph_constrain_env_contract():
    from gsmarl_amd import MultiAgentGraphConstrainEnv, make_env
    env = make_env("navigation", "MultiAgentGraphConstrainEnv", device=DEV, n_agents=3, n_envs=1)
    obs, aid, node, adj = env.reset(seed=1)
    assert len(obs) == 3 and obs[0].shape == (6,) and node[0].shape == (9, 7) and adj[0].shape == (9, 9)
    a = [np.eye(5)[k] for k in (1, 2, 3)]
    obs, aid, node, adj, rew, cost, done, info = env.step(a)
    assert isinstance(env, MultiAgentGraphConstrainEnv)
    assert len(rew) == 3 and len(cost) == 3 and done == [False] * 3 and info[0]["cost"] == cost[0]
    g = env.graph()
    ei = g["edge_index"].cpu().numpy()
    # dense adjacency carries the edge distances
    assert np.allclose(adj[0][ei[0], ei[1]], g["edge_attr"].cpu().numpy())
    vec = make_env("navigation", "MultiAgentConstrainEnv", device=DEV, n_agents=4, n_envs=8)
    o = vec.reset(seed=2)
    assert o.shape == (8, 4, 6)
    o, r, c, d, inf = vec.step(np.random.randint(0, 5, size=(8, 4)))
    assert r.shape == (8, 4, 1) and c.shape == (8, 4, 1) and d.shape == (8, 4)
