"""CPU checks of the ragged-batch oracle (oracle/ragged_ref.py): shapes,
slot geometry, assignment optimality, graph structure, and that a navigation
env inside a ragged batch is exactly the same env of a navigation batch."""
import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment as scipy_lsa

from oracle import batch_ref as br
from oracle import ragged_ref as rr


def test_env_shapes():
    cfg = rr.make_cfg(scenario="mixed", n_agents=24, n_envs=3000, seed=9, env_base=17)
    n, scn = rr.env_shapes(cfg)
    assert n.min() == 3 and n.max() == 24 and len(np.unique(n)) == 22
    assert np.array_equal(scn, (17 + np.arange(3000)) % 3)
    n2, _ = rr.env_shapes(cfg, seed=10)
    assert not np.array_equal(n, n2)
    for s in ("polygon", "line"):
        c = rr.make_cfg(scenario=s, n_agents=7, n_envs=5)
        n, scn = rr.env_shapes(c)
        assert np.all(n == 7) and np.all(scn == rr.SCENARIO_IDS[s])


def test_padded_sizes():
    assert rr.RSpec(rr.make_cfg(scenario="mixed", n_agents=24)).Emax == 72
    assert rr.RSpec(rr.make_cfg(scenario="polygon", n_agents=6)).Emax == 7
    assert rr.RSpec(rr.make_cfg(scenario="line", n_agents=6)).Emax == 8


def test_slot_geometry():
    cfg = rr.make_cfg(scenario="polygon", n_agents=12)
    c = np.array([[0.25, -1.5]], np.float32)
    s = rr.slots(cfg, rr.SCN_POLYGON, 12, c)
    assert np.allclose(np.linalg.norm(s - c, axis=1), 0.5, atol=1e-6)
    cfg = rr.make_cfg(scenario="line", n_agents=5)
    ends = np.array([[-1.0, 2.0], [3.0, -0.5]], np.float32)
    s = rr.slots(cfg, rr.SCN_LINE, 5, ends)
    assert np.array_equal(s[0], ends[0]) and np.array_equal(s[-1], ends[1])
    assert np.allclose(np.diff(s, axis=0), (ends[1] - ends[0]) / 4, atol=1e-6)
    assert np.array_equal(rr.slots(cfg, rr.SCN_LINE, 1, ends)[0], ends[0] + (ends[1] - ends[0]) * np.float32(0.5))


@pytest.mark.parametrize("scenario", ["polygon", "line"])
def test_assignment_is_scipy_optimum(scenario):
    cfg = rr.make_cfg(scenario=scenario, n_agents=16, n_envs=6, seed=2)
    st = rr.new_state(cfg)
    rs = rr.RSpec(cfg)
    for b in range(6):
        n, scn, pc = rr._compact(rs, st, b)
        sigma, C = rr.assignment(cfg, scn, n, pc)
        assert sorted(sigma.tolist()) == list(range(n))
        _, col = scipy_lsa(C.astype(np.float64))
        assert np.array_equal(sigma, col)


def test_graph_structure():
    cfg = rr.make_cfg(scenario="mixed", n_agents=12, n_envs=30, seed=4)
    st = rr.new_state(cfg)
    ob = rr.observe(cfg, st)
    rs = rr.RSpec(cfg)
    ptr, ei = ob["edge_ptr"], ob["edge_index"]
    for b in range(30):
        s, t = ei[:, ptr[b]:ptr[b + 1]] - b * rs.Emax
        key = s.astype(np.int64) * rs.Emax + t
        assert np.all(np.diff(key) > 0), "row-major, unique"
        pairs = set(zip(s.tolist(), t.tolist()))
        assert all((d, a) in pairs for a, d in pairs), "undirected"
        n, scn = int(st["n"][b]), int(st["scn"][b])
        live = set(rr.store_index(rs, scn, n).tolist())
        assert set(s.tolist()) <= live and set(t.tolist()) <= live, "no padding node in edges"
        tg = rr.n_targets(scn, n)
        for i in range(n):
            if scn == rr.SCN_NAV:
                assert (i, rs.Nmax + i) in pairs
            else:
                assert all((i, rs.Nmax + k) in pairs for k in range(tg))
        pad = [q for q in range(rs.Emax) if q not in live]
        assert np.all(ob["node_feat"][b, pad, 6] == rr.TYPE_PAD)
        assert np.all(ob["node_feat"][b, pad, :6] == 0)


def test_navigation_env_equals_navigation_batch():
    """A navigation env of N agents inside a mixed batch is env `gid` of a
    navigation batch of N: same layout, physics, reward, cost, graph."""
    cfg = rr.make_cfg(scenario="mixed", n_agents=24, n_envs=40, seed=6, episode_length=3)
    st = rr.new_state(cfg)
    rs = rr.RSpec(cfg)
    rng = np.random.default_rng(1)
    acts = rng.integers(0, 5, (4, 40, 24))
    states = [st]
    outs = []
    for t in range(4):
        st, ob = rr.step(cfg, st, acts[t], 1, np.float64)
        states.append(st)
        outs.append(ob)
    checked = 0
    for b in np.nonzero(states[0]["scn"] == rr.SCN_NAV)[0][:5]:
        n = int(states[0]["n"][b])
        ncfg = br.make_cfg(n_agents=n, n_envs=b + 1, seed=6, episode_length=3)
        nst = br.new_state(ncfg, seed=6, dtype=np.float64)
        idx = rr.store_index(rs, rr.SCN_NAV, n)
        assert np.array_equal(nst["pos"][b], states[0]["pos"][b, idx])
        for t in range(4):
            a = np.zeros((b + 1, n), np.int64)
            a[b] = acts[t][b, :n]
            nst, nob = br.step(ncfg, nst, a, 1, np.float64, seed=6)
            assert np.array_equal(nst["pos"][b], states[t + 1]["pos"][b, idx])
            assert np.array_equal(nob["reward"][b], outs[t]["reward"][b, :n])
            assert np.array_equal(nob["cost"][b], outs[t]["cost"][b, :n])
            # graph of env b, nav ids b*E + e  ->  ragged ids b*E_max + idx[e]
            s, e = nob["edge_index"][:, nob["edge_ptr"][b]:nob["edge_ptr"][b + 1]] - b * (3 * n)
            rs_, re_ = outs[t]["edge_index"][:, outs[t]["edge_ptr"][b]:outs[t]["edge_ptr"][b + 1]] - b * rs.Emax
            assert np.array_equal(idx[s], rs_) and np.array_equal(idx[e], re_)
        checked += 1
    assert checked >= 3


def test_rollout_bookkeeping():
    cfg = rr.make_cfg(scenario="mixed", n_agents=8, n_envs=9, seed=1, episode_length=4, shared_reward=True)
    st = rr.new_state(cfg)
    for t in range(9):
        st, ob = rr.step(cfg, st, np.zeros((9, 8), np.int64), 1, np.float64)
        assert np.all(ob["done"] == ((t + 1) % 4 == 0))
    assert np.all(st["episode"] == 2) and np.all(st["step"] == 1)
    n = st["n"]
    for b in range(9):
        r = ob["reward"][b]
        assert np.all(r[:n[b]] == r[0]) and np.all(r[n[b]:] == 0)
