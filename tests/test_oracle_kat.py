"""Oracle self-checks: analytic known-answer tests of the MPE semantics
(SURVEY.md §4 tier 1) and agreement of the two independent restatements
(object-per-entity ``mpe_ref`` vs vectorised ``batch_ref``)."""
import math

import numpy as np
import pytest

from oracle import batch_ref as br
from oracle import mpe_ref as mr


def _state(cfg, pos, vel=None):
    pos = np.asarray(pos, np.float64)[None]
    vel = np.zeros((1, cfg.n_agents, 2)) if vel is None else np.asarray(vel, np.float64)[None]
    return pos, vel


def softplus(z):
    return max(z, 0.0) + math.log1p(math.exp(-abs(z)))


# ---------------------------------------------------------------- analytic KATs
def test_free_flight_with_damping():
    cfg = br.make_cfg(n_agents=1, n_obstacles=0)
    pos, vel = _state(cfg, [[0.3, -0.2], [5.0, 5.0]], [[1.0, 0.0]])
    p, v = br.physics(cfg, pos, vel, np.array([[0]]), 1)
    assert v[0, 0] == pytest.approx([0.75, 0.0], abs=1e-15)
    assert p[0, 0] == pytest.approx([0.3 + 0.075, -0.2], abs=1e-15)
    p, v = br.physics(cfg, pos, vel, np.array([[1]]), 1)       # u = +5 x
    assert v[0, 0] == pytest.approx([1.25, 0.0], abs=1e-15)
    assert p[0, 0] == pytest.approx([0.3 + 0.125, -0.2], abs=1e-15)
    assert np.array_equal(p[0, 1], pos[0, 1])                  # goal immovable


def test_speed_clamp():
    cfg = br.make_cfg(n_agents=1, n_obstacles=0, max_speed=1.0)
    pos, vel = _state(cfg, [[0.0, 0.0], [5.0, 5.0]], [[0.0, 2.0]])
    p, v = br.physics(cfg, pos, vel, np.array([[0]]), 1)        # 1.5 -> 1.0
    assert v[0, 0] == pytest.approx([0.0, 1.0], abs=1e-15)
    assert p[0, 0] == pytest.approx([0.0, 0.1], abs=1e-15)


@pytest.mark.parametrize("d", [0.09, 0.1, 0.12, 0.3])
def test_two_body_head_on_contact(d):
    cfg = br.make_cfg(n_agents=2, n_obstacles=0)
    pos, vel = _state(cfg, [[-d / 2, 0.0], [d / 2, 0.0], [3, 3], [-3, -3]])
    p, v = br.physics(cfg, pos, vel, np.zeros((1, 2), int), 1)
    dmin, k, c = 0.1, 1e-3, 100.0
    f = c * k * softplus(-(d - dmin) / k)          # magnitude, pushes apart
    assert v[0, 0, 0] == pytest.approx(-f * 0.1, rel=1e-12, abs=1e-300)
    assert v[0, 1, 0] == pytest.approx(+f * 0.1, rel=1e-12, abs=1e-300)
    assert v[0, :, 1] == pytest.approx([0, 0], abs=1e-300)
    assert p[0, 0, 0] == pytest.approx(-d / 2 - f * 0.01, rel=1e-12)


def test_immovable_obstacle():
    cfg = br.make_cfg(n_agents=1, n_obstacles=1)
    # agent overlapping an obstacle: agent pushed, obstacle fixed
    pos, vel = _state(cfg, [[0.0, 0.0], [2.0, 2.0], [0.1, 0.0]])
    p, v = br.physics(cfg, pos, vel, np.zeros((1, 1), int), 1)
    f = 100.0 * 1e-3 * softplus(-(0.1 - 0.13) / 1e-3)
    assert v[0, 0, 0] == pytest.approx(-f * 0.1, rel=1e-12)
    assert np.array_equal(p[0, 2], pos[0, 2])


def test_coincident_guard():
    cfg = br.make_cfg(n_agents=2, n_obstacles=0)
    pos, vel = _state(cfg, [[0.5, 0.5], [0.5, 0.5], [1, 1], [2, 2]])
    p, v = br.physics(cfg, pos, vel, np.zeros((1, 2), int), 1)
    assert np.all(np.isfinite(p)) and np.all(v == 0)
    _, cost = br.reward_cost(cfg, pos)
    assert cost[0].tolist() == [1.0, 1.0]          # coincident agents collide


def test_coincident_strict_is_mpe_nan_and_spreads():
    """Appendix A S16 strict mode: MPE's delta/dist = 0/0 makes both agents of
    a coincident pair NaN; on the next step every pair with a NaN agent is NaN,
    so every agent of the env is; other envs are untouched. The flags follow."""
    cfg = br.make_cfg(n_agents=3, n_obstacles=1, strict_degenerate=True, n_envs=2)
    base = [[0.5, 0.5], [0.5, 0.5], [-1.0, -1.0], [1, 1], [2, 2], [0, 2], [1.5, -1.5]]
    pos = np.array([base, base], np.float64)
    pos[1, 1] = [0.9, 0.5]                              # env 1: no coincident pair
    vel = np.zeros((2, 3, 2))
    assert br.degenerate(cfg, pos).tolist() == [1, 0]
    p, v = br.physics(cfg, pos, vel, np.zeros((2, 3), int), 1)
    assert np.isnan(v[0, :2]).all() and np.isnan(p[0, :2]).all()
    assert np.isfinite(v[0, 2]).all() and np.isfinite(p[0, 2]).all() and np.isfinite(p[1]).all()
    assert br.degenerate(cfg, p).tolist() == [2, 0]
    p2, v2 = br.physics(cfg, p, v, np.zeros((2, 3), int), 1)
    assert np.isnan(v2[0]).all() and np.isfinite(v2[1]).all()
    assert np.array_equal(p2[0, 3:], pos[0, 3:])        # landmarks never move
    # the guard (default): zero contact force for the coincident pair, finite
    gcfg = br.make_cfg(n_agents=3, n_obstacles=1, n_envs=2)
    pg, vg = br.physics(gcfg, pos, vel, np.zeros((2, 3), int), 1)
    assert np.isfinite(pg).all() and np.all(vg[0, :2] == 0)
    # an agent on an obstacle is flagged too; an obstacle pair alone is not
    q = np.array([base], np.float64)
    q[0, 1] = [0.2, 0.2]
    q[0, 2] = q[0, 6]
    assert br.degenerate(gcfg, q).tolist() == [1]


def test_strict_mpe_ref_equals_batch_ref():
    cfg = br.make_cfg(n_agents=4, n_obstacles=2, strict_degenerate=True)
    env = mr.GraphConstrainEnv(cfg)
    env.reset(seed=1)
    pos = _crowd(4, 2, 0.3, 4)
    pos[3] = pos[8]                                     # agent 3 on obstacle 0
    vel = np.zeros((4, 2))
    env.set_state(pos, vel)
    st = dict(pos=pos[None].copy(), vel=vel[None].copy(), step=np.zeros(1, np.int32),
              episode=np.zeros(1, np.int32), ep_acc=np.zeros((1, 2)), ep_last=np.zeros((1, 2)))
    for t in range(3):
        a = np.array([1, 2, 3, 4])
        with np.errstate(invalid="ignore"):
            env.step(list(np.eye(5)[a]))
        st, ob = br.step(cfg, st, a[None], 1, np.float64)
        p, v = env.get_state()
        assert np.array_equal(np.isnan(p), np.isnan(st["pos"][0])), t
        assert np.allclose(p, st["pos"][0], rtol=0, atol=1e-12, equal_nan=True)
        assert np.allclose(v, st["vel"][0], rtol=0, atol=1e-12, equal_nan=True)
    assert np.isnan(p[:4]).all()                        # spread to every agent by step 2


@pytest.mark.parametrize("k,u", [(0, (0, 0)), (1, (5, 0)), (2, (-5, 0)), (3, (0, 5)), (4, (0, -5)), (7, (0, 0))])
def test_action_mapping(k, u):
    cfg = br.make_cfg(n_agents=1)
    assert br.action_force(cfg, np.array([[k]]), 1, np.float64)[0, 0].tolist() == list(u)
    if k < 5:
        oh = np.eye(5)[[k]][None]
        assert br.action_force(cfg, oh, 0, np.float64)[0, 0].tolist() == list(u)


def test_collision_predicate_strict():
    cfg = br.make_cfg(n_agents=2, n_obstacles=0)
    pos = np.array([[[0.0, 0.0], [0.1, 0.0], [1, 1], [2, 2]]])
    _, c64 = br.reward_cost(cfg, pos, np.float64)
    assert c64[0].tolist() == [0, 0]               # d == dmin -> no collision
    p32 = np.array([[[0.0, 0.0], [np.float32(0.05) + np.float32(0.05), 0.0], [1, 1], [2, 2]]], np.float32)
    _, c32 = br.reward_cost(cfg, p32, np.float32)
    assert c32[0].tolist() == [0, 0]               # d2 == dmin2 in fp32
    p32[0, 1, 0] = np.nextafter(p32[0, 1, 0], np.float32(0))
    _, c32 = br.reward_cost(cfg, p32, np.float32)
    assert c32[0].tolist() == [1, 1]


def test_edges_row_major_radius_inclusive_goal_edges():
    cfg = br.make_cfg(n_agents=2, n_obstacles=1)
    # agents 0,1 ; goals 2,3 ; obstacle 4
    pos = np.array([[[0.0, 0.0], [0.5, 0.0], [3.0, 3.0], [-3.0, 3.0], [0.0, 0.6]]], np.float32)
    ptr, ei, attr = br.edges(cfg, pos, np.float32)
    pairs = list(zip(ei[0].tolist(), ei[1].tolist()))
    # d(0,1) = 0.5 == R (inclusive); d(0,4) = 0.6 > R; d(1,4) = 0.78 > R
    assert pairs == [(0, 1), (0, 2), (1, 0), (1, 3), (2, 0), (3, 1)]
    assert ptr.tolist() == [0, 6]
    assert attr[0] == np.float32(0.5)


def test_reset_layout_box_and_determinism():
    cfg = br.make_cfg(n_agents=24, n_envs=4, seed=5)
    a = br.layout(cfg, np.arange(4), np.zeros(4, int))
    b = br.layout(cfg, np.arange(4), np.zeros(4, int))
    assert np.array_equal(a, b)
    L = np.float32(cfg.world_half)
    assert a.dtype == np.float32 and np.all(a >= -L) and np.all(a < L)
    c = br.layout(cfg, np.arange(4), np.ones(4, int))
    assert not np.array_equal(a, c)               # new episode, new layout
    d = br.layout(cfg, np.arange(1, 5), np.zeros(4, int))
    assert np.array_equal(a[1:], d[:3])           # keyed by global env id


# ------------------------------------------------- two restatements must agree
def _crowd(N, No, L, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(-L, L, size=(2 * N + No, 2))


@pytest.mark.parametrize("N,No,L,shared", [(3, 3, 0.3, False), (6, 2, 0.4, True), (12, 12, 0.8, False)])
def test_mpe_ref_equals_batch_ref(N, No, L, shared):
    cfg = br.make_cfg(n_agents=N, n_obstacles=No, shared_reward=shared, max_speed=1.5)
    env = mr.GraphConstrainEnv(cfg)
    env.reset(seed=1)
    rng = np.random.default_rng(N)
    pos = _crowd(N, No, L, N)
    vel = rng.normal(size=(N, 2))
    env.set_state(pos, vel)
    st = dict(pos=pos[None].copy(), vel=vel[None].copy(), step=np.zeros(1, np.int32),
              episode=np.zeros(1, np.int32), ep_acc=np.zeros((1, 2)), ep_last=np.zeros((1, 2)))
    for t in range(12):
        a = rng.integers(0, 5, size=N)
        _, node, ei, dist, r, c, _, info = env.step(list(np.eye(5)[a]))
        st, ob = br.step(cfg, st, a[None], 1, np.float64)
        p, v = env.get_state()
        assert np.allclose(p, st["pos"][0], rtol=0, atol=1e-12)
        assert np.allclose(v, st["vel"][0], rtol=0, atol=1e-12)
        assert np.allclose(r, ob["reward"][0], atol=1e-12)
        assert np.array_equal(np.array(c, np.float32), ob["cost"][0])
        assert [d["cost"] for d in info] == list(c)
        assert np.array_equal(ei, ob["edge_index"].astype(np.int64))
        assert np.allclose(dist, ob["edge_attr"], atol=1e-12)
        assert np.allclose(node, ob["node_feat"][0], atol=1e-12)


def test_fp32_mode_tracks_fp64_per_step():
    cfg = br.make_cfg(n_agents=24, n_envs=16)
    st = br.new_state(cfg, seed=2, dtype=np.float32)
    rng = np.random.default_rng(0)
    pos, vel = st["pos"], st["vel"]
    for t in range(20):
        a = rng.integers(0, 5, size=(16, 24))
        p32, v32 = br.physics(cfg, pos, vel, a, 1, np.float32)
        p64, v64 = br.physics(cfg, pos.astype(np.float64), vel.astype(np.float64), a, 1, np.float64)
        assert np.abs(p32 - p64).max() < 1e-6 and np.abs(v32 - v64).max() < 1e-6
        pos, vel = p32, v32


def test_episode_bookkeeping_and_auto_reset():
    cfg = br.make_cfg(n_agents=3, n_envs=2, episode_length=5)
    st = br.new_state(cfg, seed=9, dtype=np.float64)
    acc = np.zeros((2, 2))
    for t in range(1, 12):
        st, ob = br.step(cfg, st, np.zeros((2, 3), int), 1, np.float64, seed=9)
        acc += np.stack([ob["reward"].sum(-1), ob["cost"].sum(-1)], -1)
        if t % 5 == 0:
            assert ob["done"].tolist() == [1, 1]
            assert np.allclose(st["ep_last"], acc)
            acc[:] = 0
            assert st["step"].tolist() == [0, 0] and st["episode"].tolist() == [t // 5] * 2
            lay = br.layout(cfg, [0, 1], st["episode"], 9)
            assert np.array_equal(st["pos"], lay.astype(np.float64))
        else:
            assert ob["done"].tolist() == [0, 0]
