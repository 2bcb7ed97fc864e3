"""Fused rollout graphs (GSM_GRAPH_ROLL, gsm_roll_seg_kernel): all T steps of
a graph in one launch, workgroups handing the CSR edge-count prefix to each
other through tagged granules. Every state and output buffer must equal the
eager steps' (which test_gpu_parity checks against the oracle) bit for bit:
partial workgroups, auto-resets (episode length 5 and 7), all three action
formats, repeated replays (granules tagged with a launch epoch), the headline
batch (one residency round of 2048 workgroups), the reference's zero-shot
sizes 6 and 12, and the tile path's rollout (one 512-thread workgroup per env,
C3's 96 agents). The last step's edges are emitted by the rollout launch's
tail iteration (no separate emit launch). Also checked
against the CPU oracle directly at the end of a chain."""
import numpy as np
import pytest
import torch

from oracle import batch_ref as br
from parity_tol import check_state

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
KEYS = ("pos", "vel", "step_count", "episode", "node_feat", "reward", "cost", "done", "edge_count",
        "edge_ptr", "ep_acc", "ep_last", "row_mask", "contact_mask")


def _env(**kw):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    cfg = EnvConfig(**kw)
    return GpuBatchEnv(cfg, DEV), cfg


def _actions(fmt, T, B, N, gen):
    if fmt == "index":
        return torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV, generator=gen)
    if fmt == "onehot":
        k = torch.randint(0, 5, (T, B, N), device=DEV, generator=gen)
        return torch.nn.functional.one_hot(k, 5).to(torch.float32)
    return torch.rand((T, B, N, 2), device=DEV, generator=gen) * 2 - 1


def _eager(env, acts, T, seed):
    env.reset(seed=seed)
    for t in range(T):
        env.step(acts[t % acts.shape[0]], sync_edges=False)
    torch.cuda.synchronize()
    return {k: v.clone() for k, v in env.t.items()}


def _same(ref, env, what):
    for k in KEYS:
        assert torch.equal(ref[k], env.t[k]), (what, k)
    n = int(ref["edge_ptr"][-1])
    assert torch.equal(ref["edge_index"][:, :n], env.t["edge_index"][:, :n]), what
    assert torch.equal(ref["edge_attr"][:n], env.t["edge_attr"][:n]), what


@pytest.mark.parametrize("N,B,T,EL,fmt", [(24, 64, 12, 5, "index"), (24, 257, 9, 7, "index"), (24, 8, 2, 5, "index"),
                                          (24, 40, 1, 5, "index"), (24, 130, 11, 5, "onehot"), (24, 99, 8, 3, "cont"),
                                          (24, 8192, 26, 25, "index"),
                                          # C2's shape (the step kernels pack 4 envs per wave, the rollout one)
                                          (3, 64, 12, 5, "index"), (3, 4096, 15, 6, "index"), (3, 4100, 7, 3, "onehot"),
                                          (3, 333, 9, 4, "cont"),
                                          # the reference's zero-shot navigation sizes (readme.md:75)
                                          (6, 1024, 10, 4, "index"), (6, 37, 7, 3, "cont"), (12, 2048, 9, 5, "onehot"),
                                          (12, 100, 6, 4, "index"),
                                          # tile path (one workgroup per env): C3's shape
                                          (96, 16, 9, 5, "index"), (96, 33, 6, 4, "onehot"), (96, 7, 5, 2, "cont"),
                                          (96, 1024, 12, 10, "index"), (70, 9, 3, 2, "index")])
def test_roll_equals_eager(N, B, T, EL, fmt):
    env, cfg = _env(n_agents=N, n_envs=B, episode_length=EL)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(B * 31 + T)
    acts = _actions(fmt, max(T - 3, 1), B, N, gen)   # fewer action rows than steps: the ring wraps
    ref = _eager(env, acts, T, seed=11)
    env.reset(seed=11)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "roll")
    # a second replay continues from the state (granules re-zeroed by the graph)
    ref2 = {k: v.clone() for k, v in ref.items()}
    env.reset(seed=11)
    for t in range(T):
        env.step(acts[t % acts.shape[0]], sync_edges=False)
    for t in range(T):
        env.step(acts[t % acts.shape[0]], sync_edges=False)
    torch.cuda.synchronize()
    ref2 = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=11)
    env.replay(0)
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref2, env, "roll x2")
    env.close()


@pytest.mark.parametrize("N,B", [(24, 300), (96, 20), (3, 4100)])
def test_roll_emit_after_chain(N, B):
    """The bound edge-sum half holds the last step's sums after a rollout
    graph: an emit-only graph right after it re-emits the same edges."""
    T = 10
    env, cfg = _env(n_agents=N, n_envs=B, episode_length=6)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    ref = _eager(env, acts, T, seed=4)
    env.reset(seed=4)
    env.capture(acts, T, slot=1, kernels="roll")
    env.replay(1)
    env.t["edge_index"].zero_()
    env.capture(None, 1, slot=3, kernels="emit")
    env.replay(3)
    torch.cuda.synchronize()
    _same(ref, env, "roll + emit")
    env.close()


@pytest.mark.parametrize("N,B", [(24, 48), (96, 12), (6, 40), (12, 40)])
def test_roll_oracle_direct(N, B):
    """The last step of a rollout graph vs the fp64 CPU oracle stepped from
    the identical fp32 pre-step state (eager steps reach it bit for bit):
    positions/velocities within the 1e-6 bar, counters, costs and the CSR
    edges exact (fp32-mode oracle on the kernel's own positions). Episode
    length 6 puts an auto-reset inside the launch."""
    T = 9
    env, cfg = _env(n_agents=N, n_envs=B, episode_length=6, seed=21)
    ocfg = br.make_cfg(**{k: v for k, v in cfg.to_dict().items() if k in br.DEFAULTS})
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=21)
    for t in range(T - 1):
        env.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    st = {k: v.detach().cpu().numpy() for k, v in env.get_state().items()}
    ref_st = dict(pos=st["pos"].astype(np.float64), vel=st["vel"].astype(np.float64),
                  step=st["step_count"], episode=st["episode"],
                  ep_acc=st["ep_acc"].astype(np.float64), ep_last=st["ep_last"].astype(np.float64))
    nst, ob = br.step(ocfg, ref_st, acts[T - 1].cpu().numpy(), 1, np.float64, seed=21)
    env.reset(seed=21)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    torch.cuda.synchronize()
    got = {k: v.detach().cpu().numpy() for k, v in env.t.items()}
    check_state(got["pos"], nst["pos"], "pos roll")
    check_state(got["vel"], nst["vel"], "vel roll")
    assert np.array_equal(got["step_count"], nst["step"])
    assert np.array_equal(got["episode"], nst["episode"])
    assert np.array_equal(got["done"].astype(bool), ob["done"].astype(bool))
    assert np.allclose(got["reward"], ob["reward"], rtol=3e-7, atol=2e-6)
    ptr, ei, attr = br.edges(ocfg, got["pos"], np.float32)
    assert np.array_equal(got["edge_ptr"], ptr)
    assert np.array_equal(got["edge_index"][:, :ptr[-1]], ei)
    env.close()


def test_roll_rejected_where_unsupported():
    """A runtime-shape segmented config (5 agents) has no rollout kernel."""
    from gsmarl_amd._lib import GsmError
    env, cfg = _env(n_agents=5, n_envs=64)
    acts = torch.randint(0, 5, (4, 64, 5), dtype=torch.int32, device=DEV)
    env.reset(seed=1)
    with pytest.raises(GsmError):
        env.capture(acts, 4, slot=0, kernels="roll")
    env.close()


@pytest.mark.parametrize("N,B", [(3, 4096), (24, 512), (96, 16)])
def test_roll_replay_after_other_work(N, B):
    """A rollout graph replayed after eager steps and a reset (the granules of
    its previous replay are still in memory: the launch epoch in their tags
    keeps them from being taken for this replay's) equals eager steps."""
    T, EL = 15, 6
    env, cfg = _env(n_agents=N, n_envs=B, episode_length=EL)
    acts = torch.randint(0, 5, (T - 3, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=11)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    for t in range(2 * T):
        env.step(acts[t % acts.shape[0]], sync_edges=False)
    env.reset(seed=11)
    for _ in range(2):   # two replays: each runs action rows j % len(acts), j < T
        for t in range(T):
            env.step(acts[t % acts.shape[0]], sync_edges=False)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=11)
    env.replay(0)
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "replay after eager work")
    env.close()


@pytest.mark.parametrize("N,B", [(24, 8192), (3, 4096), (96, 1024)])
def test_roll_episodes_match_chain(N, B):
    """Three 100-step episodes replayed back to back (auto-resets inside each
    launch, granule epochs advancing) leave every buffer exactly as the
    per-step chain does — the BASELINE shapes at full size."""
    T = 100
    env, cfg = _env(n_agents=N, n_envs=B, episode_length=T)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=5)
    env.capture(acts, T, slot=0, kernels="both")   # lagged chain (two-kernel chain on the tile path)
    for _ in range(3):
        env.replay(0)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in env.t.items()}
    env.reset(seed=5)
    env.capture(acts, T, slot=1, kernels="roll")
    assert env.graph_is_rollout(1)
    for _ in range(3):
        env.replay(1)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "3 episodes")
    env.close()


@pytest.mark.parametrize("N,B,T,mode", [(3, 100, 1, "slots"), (24, 100, 1, "bound"), (3, 100, 3, "slots"),
                                        (24, 300, 2, "bound")])
def test_roll_recycled_granules(N, B, T, mode):
    """Back-to-back envs of one shape: each capture's granules are a fresh
    allocation, usually at the address the previous env freed, whose granules
    an agent-scope load may still see after the new allocation is zeroed (a
    hipMemset's zeros did not hide them: the second env of a pair got the
    first's group sums). Each graph is replayed three times before it is
    freed; every launch takes its own epoch from one process-wide counter,
    so no left-over granule carries a tag of the next graph's launches."""
    from gsmarl_amd import GraphRolloutBuffer
    for rep in range(3):
        env, cfg = _env(n_agents=N, n_envs=B, seed=2, episode_length=6)
        ref, _ = _env(n_agents=N, n_envs=B, seed=2, episode_length=6)
        acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
        if mode == "slots":
            gb, eb = GraphRolloutBuffer(env, episode_length=T), GraphRolloutBuffer(ref, episode_length=T)
            gb.reset(seed=2)
            gb.capture(acts)
            gb.replay()
            eb.reset(seed=2)
            for t in range(T):
                eb.insert(acts[t])
            torch.cuda.synchronize()
            got, want = gb.edge_ptr, eb.edge_ptr
        else:
            env.reset(seed=2)
            env.capture(acts, T, slot=0, kernels="roll")
            env.replay(0)
            ref.reset(seed=2)
            for t in range(T):
                ref.step(acts[t], sync_edges=False)
            torch.cuda.synchronize()
            got, want = env.t["edge_ptr"], ref.t["edge_ptr"]
        assert not env.roll_gave_up()
        assert torch.equal(got, want), (rep, (got != want).nonzero().flatten()[:8].tolist())
        for _ in range(2):   # advance this graph's epoch past the next capture's first
            gb.replay() if mode == "slots" else env.replay(0)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        env.close()
        ref.close()


def test_roll_recycled_after_many_replays():
    """A graph replayed more than 4096 times (the per-capture epoch blocks of
    round 3 ran into the next capture's block there), freed, and a new
    capture at the recycled granule allocation: the new graph still equals
    eager steps, and no bounded wait gives up."""
    N, B, T = 3, 100, 2
    env, _ = _env(n_agents=N, n_envs=B, seed=4, episode_length=6)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    env.reset(seed=4)
    env.capture(acts, T, slot=0, kernels="roll")
    for _ in range(4200):
        env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    env.close()
    env, _ = _env(n_agents=N, n_envs=B, seed=4, episode_length=6)
    ref, _ = _env(n_agents=N, n_envs=B, seed=4, episode_length=6)
    env.reset(seed=4)
    env.capture(acts, T, slot=0, kernels="roll")
    env.replay(0)
    ref.reset(seed=4)
    for t in range(T):
        ref.step(acts[t], sync_edges=False)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    assert torch.equal(env.t["edge_ptr"], ref.t["edge_ptr"])
    n = int(ref.t["edge_ptr"][-1])
    assert torch.equal(env.t["edge_index"][..., :n], ref.t["edge_index"][..., :n])
    env.close()
    ref.close()


@pytest.mark.parametrize("N,B", [(24, 8192), (3, 4096), (96, 1024), (12, 100), (6, 37)])
def test_eager_one_launch_equals_two_kernels(N, B, monkeypatch):
    """gsm_step as one rollout launch of one step (GSM_EAGER_ONE_LAUNCH=1,
    where the config has a rollout kernel; the default at 6-24 agents) leaves
    every buffer exactly as the step kernel + emit kernel pair
    (GSM_EAGER_ONE_LAUNCH=0) does, over steps with auto-resets,
    in both the bound buffers and redirected outputs."""
    T, EL = 7, 5
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    envs = []
    for two in (True, False):
        if two:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "0")
        else:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "1")
        env, _ = _env(n_agents=N, n_envs=B, episode_length=EL, seed=9)
        env.reset(seed=9)
        for t in range(T):
            env.step(acts[t], sync_edges=False)   # the first step decides the handle's path
        envs.append(env)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in envs[0].t.items()}
    _same(ref, envs[1], "eager one launch")
    for e in envs:
        assert not e.roll_gave_up()
        e.close()


@pytest.mark.parametrize("N,B", [(24, 512), (96, 16), (12, 100)])
def test_eager_one_launch_redirected_outputs(N, B, monkeypatch):
    """The one-launch eager step (GSM_EAGER_ONE_LAUNCH=1) writing every output
    into a fresh redirected set per step (gsm_step_into: node features,
    reward, cost, done, counts, CSR pointers and edges) gives exactly the
    two-kernel pair's outputs of every step, auto-resets included."""
    T, EL = 6, 4
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    keys = ("node_feat", "reward", "cost", "done", "edge_count", "edge_ptr")
    got = []
    for two in (True, False):
        if two:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "0")
        else:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "1")
        env, _ = _env(n_agents=N, n_envs=B, episode_length=EL, seed=13)
        env.reset(seed=13)
        steps = []
        for t in range(T):
            out = {k: torch.full_like(env.t[k], -7) for k in keys}
            out["edge_index"] = torch.full_like(env.t["edge_index"], -7)
            out["edge_attr"] = torch.full_like(env.t["edge_attr"], -7.0)
            env.step(acts[t], out=out)
            steps.append(out)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        got.append(steps)
        env.close()
    for t, (a, b) in enumerate(zip(*got)):
        for k in keys:
            assert torch.equal(a[k], b[k]), (t, k)
        n = int(a["edge_ptr"][-1])
        assert torch.equal(a["edge_index"][:, :n], b["edge_index"][:, :n]), t
        assert torch.equal(a["edge_attr"][:n], b["edge_attr"][:n]), t


def test_roll_capture_refuses_action_rows_past_4gib():
    """The rollout kernels address the action rows with 32-bit byte offsets:
    an explicit GSM_GRAPH_ROLL capture whose rows span 4 GiB or more is
    refused (GSM_EINVAL) before anything is launched; the default capture
    takes the per-step chain instead (no launch here either: nothing replays)."""
    import ctypes as C

    from gsmarl_amd import _lib
    env, _ = _env(n_agents=24, n_envs=64, episode_length=4)
    acts = torch.zeros((2, 64, 24), dtype=torch.int32, device=DEV)
    ptr = C.c_void_p(acts.data_ptr())
    rc = env.lib.gsm_graph_capture(env._h, 0, ptr, 1 << 31, 2, 2, _lib.ACT_INDEX, _lib.GRAPH_ROLL)
    assert rc == _lib.GSM_EINVAL
    assert "4 GiB" in _lib.last_error(env.lib, env._h)
    rc = env.lib.gsm_graph_capture(env._h, 0, ptr, 1 << 31, 2, 2, _lib.ACT_INDEX, 0)
    assert rc == _lib.GSM_OK, _lib.last_error(env.lib, env._h)
    assert not env.graph_is_rollout(0)
    env.close()


@pytest.mark.parametrize("N,B", [(24, 256), (12, 100)])
def test_eager_captured_steps_between_one_launch_steps(N, B, monkeypatch):
    """env.step inside a torch.cuda.graph capture records the one-launch step
    (its hand-off epoch and chunk-sum half live in device memory and the
    kernel advances them, so every replay takes a fresh epoch); replays of
    such a graph interleaved with the default one-launch eager steps leave
    every buffer as the same sequence run with two launches everywhere
    (GSM_EAGER_ONE_LAUNCH=0), auto-resets included."""
    T, EL = 9, 4
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    got = []
    for two in (True, False):
        if two:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "0")
        else:
            monkeypatch.delenv("GSM_EAGER_ONE_LAUNCH", raising=False)
        env, _ = _env(n_agents=N, n_envs=B, episode_length=EL, seed=5)
        env.reset(seed=5)
        static = acts[0].clone()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=DEV)
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                env.step(static, sync_edges=False)   # recorded, not run
        torch.cuda.synchronize()
        for t in range(T):
            if t % 3 == 1:
                static.copy_(acts[t])
                g.replay()
            else:
                env.step(acts[t], sync_edges=False)
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        got.append({k: v.clone() for k, v in env.t.items()})
        del g
        env.close()
    ref = got[0]
    for k in KEYS:
        assert torch.equal(ref[k], got[1][k]), k
    n = int(ref["edge_ptr"][-1])
    assert torch.equal(ref["edge_index"][:, :n], got[1]["edge_index"][:, :n])
    assert torch.equal(ref["edge_attr"][:n], got[1]["edge_attr"][:n])


def test_roll_replay_refused_inside_stream_capture():
    """A rollout graph takes its own hand-off epoch and its half of the chunk-
    sum double buffer at every launch, so a launch recorded into the caller's
    stream capture (torch.cuda.graph around env.replay) would replay one of
    each every time: gsm_graph_launch refuses it (GSM_ESTATE) instead, and
    the env still steps correctly afterwards."""
    from gsmarl_amd._lib import GsmError
    N, B, T = 24, 64, 6
    env, _ = _env(n_agents=N, n_envs=B, episode_length=5)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    ref = _eager(env, acts, T, seed=3)
    env.reset(seed=3)
    env.capture(acts, T, slot=0, kernels="roll")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=DEV)
    refused = False
    with torch.cuda.stream(s):
        try:
            with torch.cuda.graph(g, stream=s):
                try:
                    env.replay(0)
                except GsmError as e:
                    refused = "stream capture" in str(e)
        except Exception:   # an empty capture may be rejected by torch itself
            pass
    assert refused
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "roll after a refused capture")
    env.close()


def test_roll_replay_after_its_stream_was_destroyed():
    """Rollout launches of one handle are ordered across streams by an event
    recorded behind each launch (no host sync, nothing held of the previous
    stream): a replay on a raw HIP stream that is destroyed right after, then
    replays on torch's stream, equal eager steps."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    N, B, T = 24, 512, 7
    env, _ = _env(n_agents=N, n_envs=B, episode_length=5)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    ref = _eager(env, acts, 3 * T, seed=8)
    env.reset(seed=8)
    env.capture(acts, T, slot=0, kernels="roll")
    torch.cuda.synchronize()
    st = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    env._chk(env.lib.gsm_graph_launch(env._h, 0, st), "gsm_graph_launch")
    assert hip.hipStreamDestroy(st) == 0
    env.replay(0)
    env.replay(0)
    torch.cuda.synchronize()
    assert not env.roll_gave_up()
    _same(ref, env, "roll across streams")
    env.close()


def _greedy(o):
    """the bench's closed-loop policy (int32 arithmetic): the discrete action
    along the larger component of (goal - position)"""
    dx, dy = o[..., 4], o[..., 5]
    ax = 2 - (dx > 0).to(torch.int32)
    ay = 4 - (dy > 0).to(torch.int32)
    return torch.where(dx.abs() > dy.abs(), ax, ay)


@pytest.mark.parametrize("N,B", [(24, 8192), (6, 300)])
def test_captured_policy_step_replays(N, B, monkeypatch):
    """The runner's captured step: one torch.cuda.graph holding the policy on
    the current observation and env.step (the one-launch step, device-side
    epoch) replayed back to back and interleaved with eager steps — three
    replays in a row, then alternating — leaves every buffer, every step's
    edges included, exactly as the same closed loop run with two launches per
    step (GSM_EAGER_ONE_LAUNCH=0), auto-resets included."""
    T, EL = 10, 4
    pattern = "GGGEGEGGEG"   # G: graph replay, E: eager policy + step
    got = []
    for two in (True, False):
        if two:
            monkeypatch.setenv("GSM_EAGER_ONE_LAUNCH", "0")
        else:
            monkeypatch.delenv("GSM_EAGER_ONE_LAUNCH", raising=False)
        env, _ = _env(n_agents=N, n_envs=B, episode_length=EL, seed=17)
        env.reset(seed=17, sync_edges=False)
        obs = env.t["node_feat"][:, :N, :6]
        side = torch.cuda.Stream(device=DEV)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _greedy(obs)   # (warm the policy's kernels; no step)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            env.step(_greedy(obs), sync_edges=False)   # recorded, not run
        steps = []
        for c in pattern[:T]:
            if c == "G":
                g.replay()
            else:
                env.step(_greedy(obs), sync_edges=False)
            steps.append({k: env.t[k].clone() for k in ("edge_ptr", "reward", "cost", "done")} |
                         {"edges": env.t["edge_index"][:, :int(env.t["edge_ptr"][-1])].clone()})
        torch.cuda.synchronize()
        assert not env.roll_gave_up()
        got.append(({k: v.clone() for k, v in env.t.items()}, steps))
        del g
        env.close()
    (ref, ref_steps), (one, one_steps) = got
    for k in KEYS:
        assert torch.equal(ref[k], one[k]), k
    for t, (a, b) in enumerate(zip(ref_steps, one_steps)):
        for k in a:
            assert torch.equal(a[k], b[k]), (t, k)


@pytest.mark.parametrize("N,B", [(24, 8193), (96, 1025)])
def test_roll_capture_refuses_past_one_residency_round(N, B):
    """A batch past one residency round of its rollout kernel (8192 envs of
    the one-env-per-wave rollout: 2048 workgroups, the one-hop prefix's 64 x
    64; 1024 of the tile rollout) is refused by an explicit GSM_GRAPH_ROLL
    capture (GSM_EINVAL, gsm.h) before anything launches; the default capture
    takes the per-step chain, which equals eager steps."""
    import ctypes as C

    from gsmarl_amd import _lib
    T = 3
    env, _ = _env(n_agents=N, n_envs=B, episode_length=2)
    acts = torch.randint(0, 5, (T, B, N), dtype=torch.int32, device=DEV)
    ptr = C.c_void_p(acts.data_ptr())
    stride = acts[0].numel() * 4
    rc = env.lib.gsm_graph_capture(env._h, 0, ptr, stride, T, T, _lib.ACT_INDEX, _lib.GRAPH_ROLL)
    assert rc == _lib.GSM_EINVAL
    assert "residency round" in _lib.last_error(env.lib, env._h)
    ref = _eager(env, acts, T, seed=6)
    env.reset(seed=6)
    env.capture(acts, T, slot=0, kernels="both")
    assert not env.graph_is_rollout(0)
    env.replay(0)
    torch.cuda.synchronize()
    _same(ref, env, "chain past one residency round")
    env.close()


def test_captured_multi_step_policy_graph():
    """A graph holding three policy + env.step iterations (a runner capturing
    a stretch of its rollout: three one-launch step nodes, each taking the
    epoch the previous one advanced on the device) replayed three times
    equals nine two-launch steps of the same closed loop, auto-resets
    included."""
    import os
    N, B, S, R, EL = 24, 1024, 3, 3, 4
    got = []
    for two in (True, False):
        if two:
            os.environ["GSM_EAGER_ONE_LAUNCH"] = "0"
        try:
            env, _ = _env(n_agents=N, n_envs=B, episode_length=EL, seed=23)
            env.reset(seed=23, sync_edges=False)
            obs = env.t["node_feat"][:, :N, :6]
            if two:
                for _ in range(S * R):
                    env.step(_greedy(obs), sync_edges=False)
            else:
                side = torch.cuda.Stream(device=DEV)
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    _greedy(obs)
                torch.cuda.current_stream().wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(S):
                        env.step(_greedy(obs), sync_edges=False)
                for _ in range(R):
                    g.replay()
            torch.cuda.synchronize()
            assert not env.roll_gave_up()
            got.append({k: v.clone() for k, v in env.t.items()})
            env.close()
        finally:
            os.environ.pop("GSM_EAGER_ONE_LAUNCH", None)
    for k in KEYS:
        assert torch.equal(got[0][k], got[1][k]), k
    n = int(got[0]["edge_ptr"][-1])
    assert torch.equal(got[0]["edge_index"][:, :n], got[1]["edge_index"][:, :n])
