"""Ragged-batch restatement: navigation / polygon / line envs of varying N in
one padded batch.

TEST INFRASTRUCTURE ONLY (the checker); see oracle/batch_ref.py's header for
the parity status (unpinned w.r.t. the true GS-MARL numerics: the scenario
files ``simple_formation.py`` / ``simple_line.py``, GSMARL.egg-info/
SOURCES.txt:24-25, are absent). What is pinned: the per-step assignment is
scipy's linear_sum_assignment (oracle/lsa_ref.py, checked against scipy
itself), and a navigation env inside a ragged batch equals the same env of a
plain navigation batch (checked in tests/test_ragged_ref.py).

Scenario contract (readme.md:89-90 + SURVEY.md Appendix A S12/S13 +
DESIGN.md §3 [DECISION]s):

* navigation (0): N agents, N goals (non-colliding), N obstacles (immovable,
  colliding); reward -|p_i - g_i|; exactly batch_ref's semantics.
* polygon (1): N agents + 1 landmark (non-colliding) at the centre of a
  regular N-gon of radius ``formation_radius`` (0.5); slot j = c + r*(cos,
  sin)(2*pi*j/N). Every step C[i][j] = |p_i - slot_j| (fp32), sigma =
  linear_sum_assignment(C), reward_i = -C[i][sigma_i].
* line (2): N agents + 2 landmarks (non-colliding); slot j = l0 + (l1 - l0) *
  t_j, t_j = j/(N-1) (0.5 if N == 1); reward as polygon.
* cost (all): number of colliders j != i with |p_i - p_j| < s_i + s_j
  (colliders = agents, plus obstacles in navigation).
* graph: radius edges (0 < d <= R) among colliders, plus agent <-> each of
  its targets (own goal / the centre / both endpoints) regardless of
  distance; node features [v, p, target - p, type] with target = own goal or
  assigned slot; type 0 agent, 1 landmark/goal, 2 obstacle, -1 padding.
* mixed (3): scenario = global env id mod 3; N_env = n_min + floor(x *
  (n_max - n_min + 1) / 2^32), x = Philox(seed; counter 0, 0, env id,
  TAG_SHAPE)[0]. Layout half-width per env sqrt(N_env/3) (or world_half > 0).

Padded storage (per env, E_max rows): agents [0, N_max), targets
[N_max, N_max + T_max), obstacles [N_max + T_max, E_max). Layout draws use
the env's compact entity index (agents, targets, obstacles), so a navigation
env of N agents lays out exactly like env ``gid`` of a navigation batch of N.
"""
from __future__ import annotations

import math

import numpy as np

from . import batch_ref as br
from .lsa_ref import linear_sum_assignment
from .philox import TAG_LAYOUT, philox4x32_10, u01_f32

SCN_NAV, SCN_POLYGON, SCN_LINE, SCN_MIXED = 0, 1, 2, 3
SCENARIO_IDS = {"navigation": SCN_NAV, "polygon": SCN_POLYGON, "line": SCN_LINE, "mixed": SCN_MIXED}
TAG_SHAPE = 2
TYPE_PAD = -1

RAGGED_DEFAULTS = dict(n_agents_min=3, formation_radius=0.5)


def make_cfg(**kw):
    """Config namespace for a ragged batch (scenario polygon/line/mixed)."""
    d = dict(br.DEFAULTS)
    d.update(RAGGED_DEFAULTS)
    d.update(kw)
    scn = SCENARIO_IDS[d["scenario"]] if isinstance(d["scenario"], str) else int(d["scenario"])
    d["scenario"] = scn
    if d["n_obstacles"] is None:
        d["n_obstacles"] = d["n_agents"] if scn == SCN_MIXED else 0
    if d["world_half"] is None:
        d["world_half"] = 0.0       # per-env sqrt(N_env / 3)
    if scn != SCN_MIXED:
        d["n_agents_min"] = d["n_agents"]
    from types import SimpleNamespace
    return SimpleNamespace(**d)


class RSpec:
    """Padded sizes of a ragged batch."""

    def __init__(self, cfg):
        self.scn = int(cfg.scenario)
        self.Nmax = int(cfg.n_agents)
        self.Tmax = {SCN_POLYGON: 1, SCN_LINE: 2}.get(self.scn, self.Nmax)
        self.Omax = self.Nmax if self.scn == SCN_MIXED else 0
        self.Emax = self.Nmax + self.Tmax + self.Omax
        self.Mmax = self.Nmax + self.Omax


def env_shapes(cfg, seed=None):
    """(N_env [B] int32, scenario [B] int32) of the batch's envs."""
    seed = int(cfg.seed if seed is None else seed)
    gids = (int(cfg.env_base) + np.arange(int(cfg.n_envs), dtype=np.int64)).astype(np.uint64)
    if int(cfg.scenario) != SCN_MIXED:
        B = int(cfg.n_envs)
        return np.full(B, int(cfg.n_agents), np.int32), np.full(B, int(cfg.scenario), np.int32)
    x0, _, _, _ = philox4x32_10(0, 0, gids & np.uint64(0xFFFFFFFF), TAG_SHAPE,
                                seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    lo, hi = int(cfg.n_agents_min), int(cfg.n_agents)
    span = np.uint64(hi - lo + 1)
    n = lo + ((x0.astype(np.uint64) * span) >> np.uint64(32)).astype(np.int64)
    scn = (gids % np.uint64(3)).astype(np.int32)
    return n.astype(np.int32), scn


def half_width(cfg, n):
    """fp32 layout half-width of an env with n agents."""
    if float(cfg.world_half) > 0:
        return np.float32(cfg.world_half)
    return np.float32(math.sqrt(n / 3.0))


def n_targets(scn, n):
    return {SCN_NAV: n, SCN_POLYGON: 1, SCN_LINE: 2}[int(scn)]


def n_obstacles(scn, n):
    return n if int(scn) == SCN_NAV else 0


def store_index(rs, scn, n):
    """compact entity index -> padded storage row, for an env (scn, n)."""
    T, O = n_targets(scn, n), n_obstacles(scn, n)
    return np.concatenate([np.arange(n), rs.Nmax + np.arange(T),
                           rs.Nmax + rs.Tmax + np.arange(O)]).astype(np.int64)


def layout_env(cfg, gid, episode, n, scn, seed=None):
    """Compact fp32 positions [E_env, 2] (Philox counter = compact entity)."""
    seed = int(cfg.seed if seed is None else seed)
    E = n + n_targets(scn, n) + n_obstacles(scn, n)
    e = np.arange(E, dtype=np.uint32)
    x0, x1, _, _ = philox4x32_10(e, np.uint32(episode), np.uint32(gid & 0xFFFFFFFF), TAG_LAYOUT,
                                 seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    L = half_width(cfg, n)
    twoL = np.float32(L * np.float32(2))
    return np.stack([u01_f32(x0) * twoL - L, u01_f32(x1) * twoL - L], -1).astype(np.float32)


# ------------------------------------------------------------------ slots
def unit_circle(n):
    """fp32 (cos, sin)(2*pi*j/n), j < n, each rounded from float64 libm."""
    return np.array([[math.cos(2.0 * math.pi * j / n), math.sin(2.0 * math.pi * j / n)]
                     for j in range(n)], dtype=np.float64).astype(np.float32)


def line_t(n):
    """fp32 j/(n-1) (0.5 for n == 1)."""
    if n == 1:
        return np.array([0.5], np.float32)
    return np.array([j / (n - 1) for j in range(n)], dtype=np.float64).astype(np.float32)


def slots(cfg, scn, n, targets):
    """fp32 slot positions [n, 2] from the env's target positions."""
    targets = np.asarray(targets, np.float32)
    if scn == SCN_POLYGON:
        r = np.float32(cfg.formation_radius)
        off = (r * unit_circle(n)).astype(np.float32)
        return (targets[0][None, :] + off).astype(np.float32)
    if scn == SCN_LINE:
        l0, l1 = targets[0], targets[1]
        t = line_t(n)[:, None]
        return (l0[None, :] + (l1 - l0)[None, :] * t).astype(np.float32)
    raise ValueError(scn)


def assignment(cfg, scn, n, pos_c):
    """(sigma [n] int64, C [n, n] fp32) on an env's compact fp32 positions."""
    pa = np.asarray(pos_c[:n], np.float32)
    s = slots(cfg, scn, n, pos_c[n:n + n_targets(scn, n)])
    dx = pa[:, None, 0] - s[None, :, 0]
    dy = pa[:, None, 1] - s[None, :, 1]
    C = np.sqrt(dx * dx + dy * dy).astype(np.float32)
    if not np.isfinite(pa).all():
        # Appendix A S16 (strict mode / caller-written NaN state): scipy raises
        # on such a matrix; the contract is no assignment (-1) and a NaN cost
        return np.full(n, -1, np.int64), C
    return linear_sum_assignment(C.astype(np.float64)), C


# ------------------------------------------------------------- per env
def _nav_cfg(cfg, n, No):
    kw = {k: getattr(cfg, k) for k in br.DEFAULTS if hasattr(cfg, k)}
    kw.update(n_agents=n, n_obstacles=No, n_envs=1, scenario="navigation")
    kw["world_half"] = float(half_width(cfg, n))
    return br.make_cfg(**kw)


def _as_nav_layout(scn, n, pos_c):
    """Compact positions in batch_ref's entity order (agents, goals,
    obstacles); polygon/line get zero dummy goals (ignored by physics)."""
    if scn == SCN_NAV:
        return pos_c
    return np.concatenate([pos_c[:n], np.zeros((n, 2), pos_c.dtype)])


def physics_env(cfg, scn, n, pos_c, vel, actions, fmt, dtype):
    """One World.step of one env on compact positions -> (pos_c', vel')."""
    No = n_obstacles(scn, n)
    ncfg = _nav_cfg(cfg, n, No)
    p = _as_nav_layout(scn, n, np.asarray(pos_c, dtype))[None]
    p2, v2 = br.physics(ncfg, p, np.asarray(vel, dtype)[None], np.asarray(actions)[None], fmt, dtype)
    out = np.array(pos_c, dtype=dtype, copy=True)
    out[:n] = p2[0, :n]
    return out, v2[0]


def reward_cost_env(cfg, scn, n, pos_c, dtype):
    """(reward [n], cost [n] fp32 counts, sigma or None)."""
    No = n_obstacles(scn, n)
    ncfg = _nav_cfg(cfg, n, No)
    _, cost = br.reward_cost(ncfg, _as_nav_layout(scn, n, np.asarray(pos_c, dtype))[None], dtype)
    cost = cost[0]
    if scn == SCN_NAV:
        r, _ = br.reward_cost(ncfg, np.asarray(pos_c, dtype)[None], dtype)
        r, sigma = r[0], None
    else:
        sigma, C = assignment(cfg, scn, n, np.asarray(pos_c, np.float32))
        if (sigma < 0).any():
            r = np.full(n, np.nan, dtype)
        elif np.dtype(dtype) == np.float64:
            s = slots(cfg, scn, n, np.asarray(pos_c, np.float32)[n:]).astype(np.float64)
            d = np.asarray(pos_c, np.float64)[:n] - s[sigma]
            r = -np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
        else:
            r = -C[np.arange(n), sigma]
        if cfg.shared_reward:
            r = np.full(n, r.sum(), dtype=r.dtype)
    return np.asarray(r, dtype), cost, sigma


def node_features_env(cfg, rs, scn, n, pos_c, vel, sigma):
    """Padded node-feature rows [E_max, 7] (fp32) of one env."""
    pos_c = np.asarray(pos_c, np.float32)
    nf = np.zeros((rs.Emax, br.NODE_FEAT_DIM), np.float32)
    nf[:, 6] = TYPE_PAD
    idx = store_index(rs, scn, n)
    T, O = n_targets(scn, n), n_obstacles(scn, n)
    types = np.concatenate([np.zeros(n), np.ones(T), np.full(O, 2)]).astype(np.float32)
    nf[idx, 2:4] = pos_c
    nf[idx, 6] = types
    nf[:n, 0:2] = vel
    tgt = pos_c[n:2 * n] if scn == SCN_NAV else slots(cfg, scn, n, pos_c[n:n + T])[np.maximum(sigma, 0)]
    nf[:n, 4:6] = tgt - pos_c[:n]
    return nf


def adjacency_env(cfg, scn, n, pos_c):
    """Dense compact connectivity [E_env, E_env] and fp32 d2."""
    pos_c = np.asarray(pos_c, np.float32)
    T, O = n_targets(scn, n), n_obstacles(scn, n)
    E = n + T + O
    dx = pos_c[:, None, 0] - pos_c[None, :, 0]
    dy = pos_c[:, None, 1] - pos_c[None, :, 1]
    d2 = dx * dx + dy * dy
    coll = np.concatenate([np.ones(n, bool), np.zeros(T, bool), np.ones(O, bool)])
    R = np.float32(cfg.sense_radius)
    R2 = np.float32(R * R)
    conn = (d2 > 0) & (d2 <= R2) & coll[:, None] & coll[None, :]
    conn &= ~np.eye(E, dtype=bool)
    i = np.arange(n)
    if scn == SCN_NAV:
        conn[i, n + i] = True
        conn[n + i, i] = True
    else:
        for t in range(T):
            conn[i, n + t] = True
            conn[n + t, i] = True
    return conn, d2


def degenerate_env(scn, n, pos_c):
    """Appendix A S16 flags of one env (as batch_ref.degenerate): 1 = two
    colliders, at least one an agent, at fp32 d2 = 0; 2 = a non-finite agent."""
    pos_c = np.asarray(pos_c, np.float32)
    T, O = n_targets(scn, n), n_obstacles(scn, n)
    coll = np.concatenate([pos_c[:n], pos_c[n + T:n + T + O]])
    with np.errstate(invalid="ignore", over="ignore"):
        dx = coll[:n, None, 0] - coll[None, :, 0]
        dy = coll[:n, None, 1] - coll[None, :, 1]
        d2 = dx * dx + dy * dy
    coinc = bool(((d2 == 0) & ~np.eye(n, n + O, dtype=bool)).any())
    nonfin = not np.isfinite(pos_c[:n]).all()
    return np.uint8(int(coinc) | (int(nonfin) << 1))


def edges_env(cfg, rs, scn, n, pos_c, b):
    """Row-major (storage order) edges of env b: (src, dst) global ids
    b*E_max + row, fp32 distances."""
    conn, d2 = adjacency_env(cfg, scn, n, pos_c)
    idx = store_index(rs, scn, n)
    order = np.argsort(idx, kind="stable")     # storage order == compact order
    assert np.array_equal(order, np.arange(len(idx)))
    s, t = np.nonzero(conn)
    g = b * rs.Emax
    return (g + idx[s]).astype(np.int32), (g + idx[t]).astype(np.int32), np.sqrt(d2[s, t]).astype(np.float32)


# --------------------------------------------------------------- batch
def new_state(cfg, seed=None, dtype=np.float32):
    """State after reset(seed): padded storage, episode 0 everywhere."""
    seed = int(cfg.seed if seed is None else seed)
    rs = RSpec(cfg)
    B = int(cfg.n_envs)
    n_b, scn_b = env_shapes(cfg, seed)
    pos = np.zeros((B, rs.Emax, 2), dtype)
    for b in range(B):
        pos[b, store_index(rs, scn_b[b], n_b[b])] = layout_env(cfg, int(cfg.env_base) + b, 0,
                                                               n_b[b], scn_b[b], seed)
    return dict(pos=pos, vel=np.zeros((B, rs.Nmax, 2), dtype), step=np.zeros(B, np.int32),
                episode=np.zeros(B, np.int32), ep_acc=np.zeros((B, 2), np.float64),
                ep_last=np.zeros((B, 2), np.float64), n=n_b, scn=scn_b, seed=seed)


def _compact(rs, st, b):
    n, scn = int(st["n"][b]), int(st["scn"][b])
    return n, scn, st["pos"][b, store_index(rs, scn, n)]


def observe(cfg, st, dtype=np.float32):
    """node_feat, assign, edges on the current layout (fp32 positions)."""
    rs = RSpec(cfg)
    B = st["pos"].shape[0]
    nf = np.zeros((B, rs.Emax, br.NODE_FEAT_DIM), np.float32)
    assign = np.full((B, rs.Nmax), -1, np.int32)
    deg = np.zeros(B, np.uint8)
    src, dst, attr, counts = [], [], [], np.zeros(B, np.int64)
    for b in range(B):
        n, scn, pc = _compact(rs, st, b)
        pc32 = np.asarray(pc, np.float32)
        deg[b] = degenerate_env(scn, n, pc32)
        sigma = None
        if scn != SCN_NAV:
            sigma, _ = assignment(cfg, scn, n, pc32)
            assign[b, :n] = sigma
        nf[b] = node_features_env(cfg, rs, scn, n, pc32, np.asarray(st["vel"][b, :n], np.float32), sigma)
        s, t, a = edges_env(cfg, rs, scn, n, pc32, b)
        src.append(s)
        dst.append(t)
        attr.append(a)
        counts[b] = len(s)
    ptr = np.zeros(B + 1, np.int64)
    np.cumsum(counts, out=ptr[1:])
    ei = np.stack([np.concatenate(src), np.concatenate(dst)]).astype(np.int32) if B else np.zeros((2, 0), np.int32)
    return dict(node_feat=nf, assign=assign, edge_ptr=ptr, edge_index=ei,
                edge_attr=np.concatenate(attr) if B else np.zeros(0, np.float32), degenerate=deg)


def step(cfg, st, actions, fmt=1, dtype=np.float64):
    """One env.step of the ragged batch (same episode/auto-reset convention
    as batch_ref.step). ``actions`` are padded [B, N_max(, k)]; the extra
    agents' entries are ignored. Returns (new_state, outputs)."""
    rs = RSpec(cfg)
    st = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in st.items()}
    st["pos"] = st["pos"].astype(dtype)
    st["vel"] = st["vel"].astype(dtype)
    B = st["pos"].shape[0]
    reward = np.zeros((B, rs.Nmax), dtype)
    cost = np.zeros((B, rs.Nmax), np.float32)
    done = np.zeros(B, np.uint8)
    actions = np.asarray(actions)
    for b in range(B):
        n, scn, pc = _compact(rs, st, b)
        idx = store_index(rs, scn, n)
        pc2, v2 = physics_env(cfg, scn, n, pc, st["vel"][b, :n], actions[b, :n], fmt, dtype)
        st["pos"][b, idx] = pc2
        st["vel"][b, :n] = v2
        r, c, _ = reward_cost_env(cfg, scn, n, pc2, dtype)
        reward[b, :n] = r
        cost[b, :n] = c
        st["step"][b] += 1
        st["ep_acc"][b] += [float(np.asarray(r, np.float64).sum()), float(c.astype(np.float64).sum())]
        if st["step"][b] >= int(cfg.episode_length):
            done[b] = 1
            if cfg.auto_reset:
                st["ep_last"][b] = st["ep_acc"][b]
                st["ep_acc"][b] = 0
                st["episode"][b] += 1
                st["step"][b] = 0
                st["pos"][b, idx] = layout_env(cfg, int(cfg.env_base) + b, int(st["episode"][b]), n, scn,
                                               st["seed"])
                st["vel"][b, :n] = 0
    ob = observe(cfg, st, dtype)
    ob.update(reward=reward, cost=cost, done=done)
    return st, ob
