"""Fused rollout of ragged batches (polygon / line / mixed; config C4):
gsm_roll_ragged_kernel runs all T steps of a graph in one launch, one env per
wave, each env packing its edges `depth` steps behind its own step through a
per-env slab. Every state and output buffer must equal the
eager steps' bit for bit (which test_gpu_ragged checks against the oracle):
partial workgroups, auto-resets inside the launch, all three action formats,
pack depths 2..8, repeated replays, rollout-buffer slots (assignments
included), three full-size C4 episodes against the lagged chain (envs dealt
to the SIMDs by cost), and the last step of a launch against
oracle/ragged_ref.py directly."""
import os

import numpy as np
import pytest
import torch

from oracle import ragged_ref as rr
from parity_tol import check_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
KEYS = ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "done", "edge_count",
        "edge_ptr", "ep_acc", "ep_last", "row_mask", "assign", "env_shape", "lsa_v", "lsa_col", "lsa_stats")


def _env(**kw):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    return GpuBatchEnv(EnvConfig(**kw), DEV)


def _acts(fmt, T, B, N, gen):
    if fmt == "index":
        return torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV, generator=gen)
    if fmt == "onehot":
        k = torch.randint(0, 5, (T, B, N), device=DEV, generator=gen)
        return torch.nn.functional.one_hot(k, 5).to(torch.float32)
    return torch.rand((T, B, N, 2), device=DEV, generator=gen) * 2 - 1


def _same(ref, env, what):
    for k in KEYS:
        assert torch.equal(ref[k], env.t[k]), (what, k)
    n = int(ref["edge_ptr"][-1])
    assert torch.equal(ref["edge_index"][:, :n], env.t["edge_index"][:, :n]), what
    assert torch.equal(ref["edge_attr"][:n], env.t["edge_attr"][:n]), what


def _fresh(env, seed):
    """reset(seed) and an empty assignment warm-start cache (the cache is not
    reset by env.reset: equal runs must start from equal caches)"""
    env.reset(seed=seed)
    env.t["lsa_v"].zero_()
    env.t["lsa_col"].fill_(-1)
    env.t["lsa_stats"].zero_()


@pytest.fixture
def depth(request):
    old = os.environ.get("GSM_ROLL_DEPTH")
    if request.param is not None:
        os.environ["GSM_ROLL_DEPTH"] = str(request.param)
    yield request.param
    if old is None:
        os.environ.pop("GSM_ROLL_DEPTH", None)
    else:
        os.environ["GSM_ROLL_DEPTH"] = old


@pytest.mark.parametrize("depth,scenario,N,B,T,EL,fmt", [
    (None, "mixed", 24, 257, 9, 3, "index"), (None, "mixed", 24, 64, 2, 5, "index"),
    (None, "mixed", 24, 40, 1, 5, "index"), (None, "polygon", 12, 130, 7, 4, "onehot"),
    (None, "line", 9, 64, 5, 3, "cont"), (None, "mixed", 24, 8192, 12, 5, "index"),
    (None, "mixed", 24, 4096, 6, 4, "onehot"),
    (2, "mixed", 24, 300, 11, 4, "index"), (8, "mixed", 24, 300, 11, 4, "index"), (8, "polygon", 24, 100, 3, 2, "index"),
], indirect=["depth"])
def test_roll_ragged_equals_eager(depth, scenario, N, B, T, EL, fmt):
    env = _env(scenario=scenario, n_agents=N, n_envs=B, seed=7, episode_length=EL)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(B + T)
    acts = _acts(fmt, max(T - 2, 1), B, N, gen)   # fewer action rows than steps: the ring wraps
    _fresh(env, 7)
    for t in range(2 * T):   # each replay of the graph starts at action row 0
        env.step(acts[(t % T) % acts.shape[0]], sync_edges=False)
        if t == T - 1:
            torch.cuda.synchronize()
            ref1 = {k: v.clone() for k, v in env.t.items()}
    torch.cuda.synchronize()
    ref2 = {k: v.clone() for k, v in env.t.items()}
    _fresh(env, 7)
    env.capture(acts, T, slot=0, kernels="roll")
    assert env.graph_is_rollout(0)
    env.t["edge_index"].fill_(-7)
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref1, env, "roll")
    env.replay(0)   # a second replay continues from the state (granules of a new epoch)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref2, env, "roll x2")
    env.close()


def test_roll_ragged_recycled_granules():
    """Envs of one shape created back to back (the granules of each capture
    usually land where the previous env's were freed), each graph replayed
    three times before it is freed: the next capture's launches never take a
    left-over granule for theirs (every capture starts at a fresh block of
    launch epochs; with consecutive start epochs the second graph got the
    first's second-replay group sums)."""
    B, N, T = 300, 24, 11
    for rep in range(3):
        env = _env(scenario="mixed", n_agents=N, n_envs=B, seed=7, episode_length=4)
        acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
        _fresh(env, 7)
        for t in range(T):
            env.step(acts[t], sync_edges=False)
        torch.cuda.synchronize()
        ref = {k: v.clone() for k, v in env.t.items()}
        _fresh(env, 7)
        env.capture(acts, T, slot=0, kernels="roll")
        env.replay(0)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        _same(ref, env, f"rep {rep}")
        env.replay(0)
        env.replay(0)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        env.close()


def test_roll_ragged_episodes_match_chain():
    """C4 at full size (mixed N in {3..24} x 8192): three 100-step episodes
    replayed back to back as rollout launches leave every buffer exactly as
    the lagged per-step chain does."""
    B, N, T = 8192, 24, 100
    env = _env(scenario="mixed", n_agents=N, n_envs=B, n_agents_min=3, seed=5, episode_length=T)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    _fresh(env, 5)
    env.capture(acts, T, slot=0, kernels="both")
    for _ in range(3):
        env.replay(0)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in env.t.items()}
    _fresh(env, 5)
    env.capture(acts, T, slot=1, kernels="roll")
    assert env.graph_is_rollout(1)
    env.roll_placement()
    for _ in range(3):
        env.replay(1)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "3 episodes")
    # on an idle GPU every launch deals its envs to the SIMDs by cost
    assert env.roll_placement() == (3, 0)
    env.close()


def test_roll_ragged_xcd_dealing_same_outputs(monkeypatch):
    """The placement table only schedules: envs dealt per XCD (contiguous env
    blocks, the default) and by one cost order over the grid
    (GSM_PLACE_XCD=0) leave every buffer identical after a full-size C4
    launch, and both launches are dealt (not the identity fallback)."""
    B, N, T = 8192, 24, 30
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    out = {}
    for xcd in ("1", "0"):
        monkeypatch.setenv("GSM_PLACE_XCD", xcd)   # read when the env draws its shapes (reset)
        env = _env(scenario="mixed", n_agents=N, n_envs=B, n_agents_min=3, seed=11, episode_length=20)
        _fresh(env, 11)
        env.capture(acts, T, slot=0, kernels="roll")
        env.roll_placement()
        env.replay(0)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        assert env.roll_placement() == (1, 0), xcd
        out[xcd] = {k: v.clone() for k, v in env.t.items()}
        env.close()
    ref = out["0"]
    for k in KEYS:
        assert torch.equal(ref[k], out["1"][k]), k
    n = int(ref["edge_ptr"][-1])
    assert torch.equal(ref["edge_index"][:, :n], out["1"]["edge_index"][:, :n])
    assert torch.equal(ref["edge_attr"][:n], out["1"]["edge_attr"][:n])


@pytest.mark.parametrize("scenario,N,B", [("mixed", 24, 96), ("polygon", 10, 40), ("line", 7, 40)])
def test_roll_ragged_last_step_oracle(scenario, N, B):
    """The last step of a rollout launch vs oracle/ragged_ref.py stepped from
    the identical fp32 state before it (eager steps reach that state bit for
    bit): positions / velocities within the 1e-6 bar, edges, assignments,
    costs and node features exact. Episode length 4 puts auto-resets inside
    the launch."""
    from gsmarl_amd import EnvConfig
    T = 9
    cfg = EnvConfig(scenario=scenario, n_agents=N, n_envs=B, seed=21, episode_length=4)
    keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
    rcfg = rr.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in keys})
    env = _env(**cfg.to_dict())
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=21)
    for t in range(T - 1):
        env.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    sh = env.t["env_shape"].cpu().numpy()
    st = dict(pos=env.t["pos"].cpu().numpy(), vel=env.t["vel"].cpu().numpy(),
              step=env.t["step_count"].cpu().numpy().copy(), episode=env.t["episode"].cpu().numpy().copy(),
              ep_acc=env.t["ep_acc"].cpu().numpy().astype(np.float64),
              ep_last=env.t["ep_last"].cpu().numpy().astype(np.float64), n=sh & 0xFF, scn=sh >> 8, seed=21)
    nst, _ = rr.step(rcfg, st, acts[T - 1].cpu().numpy(), 1, np.float64)
    env.reset(seed=21)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    check_state(env.t["pos"].cpu().numpy(), nst["pos"], f"pos roll {scenario}")
    check_state(env.t["vel"].cpu().numpy(), nst["vel"], f"vel roll {scenario}")
    assert np.array_equal(env.t["step_count"].cpu().numpy(), nst["step"])
    assert np.array_equal(env.t["episode"].cpu().numpy(), nst["episode"])
    ob32 = rr.observe(rcfg, dict(st, pos=env.t["pos"].cpu().numpy(), vel=env.t["vel"].cpu().numpy(),
                                 step=nst["step"], episode=nst["episode"]))
    assert np.array_equal(env.t["edge_ptr"].cpu().numpy(), ob32["edge_ptr"])
    n = int(ob32["edge_ptr"][-1])
    assert np.array_equal(env.t["edge_index"][:, :n].cpu().numpy(), ob32["edge_index"])
    assert np.array_equal(env.t["assign"].cpu().numpy(), ob32["assign"])
    assert np.array_equal(env.t["node_feat"].cpu().numpy(), ob32["node_feat"])
    env.close()


def test_c4_full_size_sampled_oracle():
    """C4 at full size (mixed, N in {3..24} x 8192): every step of a 12-step
    run (episode length 5: auto-resets inside) checked on a sample of 85 envs
    (every 97th) against oracle/ragged_ref.py stepped from the identical fp32
    state before it — positions / velocities within the 1e-6 bar; edges,
    assignments, costs, node features and done exact — and the rollout launch
    of the same 12 steps equal to those eager steps bit for bit (its envs dealt
    to the SIMDs by cost)."""
    from gsmarl_amd import EnvConfig
    B, N, T = 8192, 24, 12
    cfg = EnvConfig(scenario="mixed", n_agents=N, n_envs=B, n_agents_min=3, seed=31, episode_length=5)
    keys = set(rr.br.DEFAULTS) | set(rr.RAGGED_DEFAULTS)
    base = {k: v for k, v in cfg.to_dict().items() if k in keys}
    env = _env(**cfg.to_dict())
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    sel = np.arange(0, B, 97)
    _fresh(env, 31)
    torch.cuda.synchronize()
    for t in range(T):
        sh = env.t["env_shape"].cpu().numpy()
        pos, vel = env.t["pos"].cpu().numpy(), env.t["vel"].cpu().numpy()
        stp, epi = env.t["step_count"].cpu().numpy(), env.t["episode"].cpu().numpy()
        acc, last = env.t["ep_acc"].cpu().numpy(), env.t["ep_last"].cpu().numpy()
        a_np = acts[t].cpu().numpy()
        env.step(acts[t], sync_edges=False)
        torch.cuda.synchronize()
        g = {k: env.t[k].cpu().numpy() for k in ("pos", "vel", "step_count", "episode", "reward", "cost", "done",
                                                 "assign", "node_feat", "edge_ptr", "edge_index", "edge_attr")}
        for b in sel:
            rcfg = rr.make_cfg(**dict(base, n_envs=1, env_base=int(b)))
            st = dict(pos=pos[b:b + 1], vel=vel[b:b + 1], step=stp[b:b + 1].copy(), episode=epi[b:b + 1].copy(),
                      ep_acc=acc[b:b + 1].astype(np.float64), ep_last=last[b:b + 1].astype(np.float64),
                      n=sh[b:b + 1] & 0xFF, scn=sh[b:b + 1] >> 8, seed=31)
            nst, out = rr.step(rcfg, st, a_np[b:b + 1], 1, np.float64)
            check_state(g["pos"][b:b + 1], nst["pos"], f"pos c4 t{t} env{b}")
            check_state(g["vel"][b:b + 1], nst["vel"], f"vel c4 t{t} env{b}")
            assert g["step_count"][b] == nst["step"][0] and g["episode"][b] == nst["episode"][0], (t, b)
            assert g["done"][b] == out["done"][0], (t, b)
            # the observation of the GPU's own fp32 positions: exact
            ob = rr.observe(rcfg, dict(st, pos=g["pos"][b:b + 1], vel=g["vel"][b:b + 1]))
            assert np.array_equal(g["assign"][b], ob["assign"][0]), (t, b)
            assert np.array_equal(g["node_feat"][b], ob["node_feat"][0]), (t, b)
            lo, hi = int(g["edge_ptr"][b]), int(g["edge_ptr"][b + 1])
            E = env.E
            assert np.array_equal(g["edge_index"][:, lo:hi] - b * E, ob["edge_index"]), (t, b)
            assert np.array_equal(g["edge_attr"][lo:hi], ob["edge_attr"]), (t, b)
            # cost / reward: the fp32 oracle on the GPU's own post-physics
            # positions (an env that reset in this step shows its new layout)
            nb, scb = int(st["n"][0]), int(st["scn"][0])
            if not g["done"][b]:
                pc = g["pos"][b, rr.store_index(rr.RSpec(rcfg), scb, nb)]
                r32, c32, _ = rr.reward_cost_env(rcfg, scb, nb, pc, np.float32)
                assert np.array_equal(g["cost"][b, :nb], c32), (t, b)
                if scb != rr.SCN_NAV:   # polygon / line: -C[i][sigma_i], exact
                    assert np.array_equal(g["reward"][b, :nb], r32), (t, b)
                else:                   # navigation: -|p - g| within fp32 rounding
                    np.testing.assert_allclose(g["reward"][b, :nb], r32, rtol=0, atol=2e-6)
    ref = {k: v.clone() for k, v in env.t.items()}
    _fresh(env, 31)
    env.capture(acts, T, slot=0, kernels="roll")
    env.roll_placement()
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "rollout vs eager at C4")
    assert env.roll_placement() == (1, 0)
    env.close()


def test_roll_ragged_into_buffer_slots():
    """capture_into on a mixed batch is one rollout launch writing slot j's
    outputs (assignments included; edges packed into slot j `depth` steps
    later); every slot equals eager step_into's."""
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
    B, N, T = 300, 24, 9
    kw = dict(scenario="mixed", n_agents=N, n_envs=B, seed=4, episode_length=4)
    env, ref = GpuBatchEnv(EnvConfig(**kw), DEV), GpuBatchEnv(EnvConfig(**kw), DEV)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    gb, eb = GraphRolloutBuffer(env, episode_length=T), GraphRolloutBuffer(ref, episode_length=T)
    gb.reset(seed=4)
    gb.capture(acts)
    assert env.graph_is_rollout(0)
    gb.replay()
    gb.validate()
    eb.reset(seed=4)
    for t in range(T):
        eb.insert(acts[t])
    torch.cuda.synchronize()
    for k in ("node_feat", "reward", "cost", "done", "edge_ptr", "edge_count", "assign"):
        assert torch.equal(getattr(gb, k), getattr(eb, k)), k
    for t in range(T + 1):
        n = int(gb.edge_ptr[t, B])
        assert torch.equal(gb.edge_index[t][:, :n], eb.edge_index[t][:, :n]), t
        assert torch.equal(gb.edge_attr[t][:n], eb.edge_attr[t][:n]), t
    env.close()
    ref.close()
