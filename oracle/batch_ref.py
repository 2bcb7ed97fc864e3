"""Vectorised NumPy restatement of the MultiAgentGraphConstrainEnv step path.

TEST INFRASTRUCTURE ONLY (the checker). The product path lives in
``gs-marl_amd/`` and never imports this package; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may.

PARITY STATUS: the reference's hot-path sources are absent from the mount
(``/root/reference/readme.md:1`` "hidden during review"; the module paths exist
only in ``GSMARL.egg-info/SOURCES.txt:14-25``) and the reference ships no tests
or fixtures. This file therefore restates the upstream MPE
semantics the reference says it modifies (``readme.md:27``) plus the contracts
stated in ``readme.md:29-41,89-90,101`` and the [DECISION]s of SURVEY.md
Appendix A. Parity with the true GS-MARL numerics is **unpinned**; the pinned
pieces are the Philox KATs (Random123), the analytic physics KATs in
``tests/test_oracle_kat.py`` and the cross-check against the independent
object-per-entity restatement ``oracle/mpe_ref.py``.

Two precision modes:

* ``np.float64`` — faithful: MPE arithmetic (``dist = sqrt(sum(delta**2))``,
  ``penetration = logaddexp(0, -(dist - dist_min)/k) * k``,
  ``force = contact_force * delta / dist * penetration``), sqrt-form predicates
  ``dist < dist_min`` (MPE ``is_collision``) and ``0 < dist <= R``
  (InforMARL ``update_graph``).
* ``np.float32`` — kernel op order for every +,-,x that feeds an integer
  output: ``d2 = dx*dx + dy*dy`` (no FMA), squared predicates
  ``d2 < dmin*dmin`` and ``0 < d2 <= R*R``. Integer outputs (cost counts,
  ``edge_index``) computed by this mode from the kernel's own fp32 positions
  must match the kernel bit for bit.

Entity order (Appendix A S4/S9): agents ``[0, N)``, goals ``[N, 2N)``,
obstacles ``[2N, 2N + No)`` — ``world.entities = agents + landmarks``.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np

from .philox import TAG_LAYOUT, philox4x32_10, u01_f32

ENT_AGENT, ENT_GOAL, ENT_OBSTACLE = 0, 1, 2
NODE_FEAT_DIM = 7   # [vx, vy, px, py, gx-px, gy-py, type]
OBS_DIM = 6         # [vx, vy, px, py, gx-px, gy-py]  (MPE order: vel, pos, goal-rel)

# Contract defaults: SURVEY.md Appendix A S2, S3, S5, S10, S11.
DEFAULTS = dict(
    scenario="navigation", n_envs=1, n_agents=3, n_obstacles=None, episode_length=100,
    auto_reset=True, shared_reward=False, env_base=0, seed=0,
    dt=0.1, damping=0.25, mass=1.0, contact_force=100.0, contact_margin=1e-3,
    sensitivity=5.0, max_speed=0.0, world_half=None,
    agent_size=0.05, goal_size=0.05, obstacle_size=0.08, sense_radius=0.5,
    strict_degenerate=False,   # Appendix A S16: MPE's NaN for a coincident pair instead of the guard
)


def make_cfg(**kw):
    """Plain config namespace with the contract defaults (duck-typed like the
    product's EnvConfig)."""
    d = dict(DEFAULTS)
    d.update(kw)
    if d["n_obstacles"] is None:
        d["n_obstacles"] = d["n_agents"]
    if d["world_half"] is None:
        d["world_half"] = float(np.sqrt(d["n_agents"] / 3.0))
    return SimpleNamespace(**d)


class Spec:
    """Derived sizes/constants. In fp32 mode every constant is formed with the
    same fp32 operations the host C code uses (``gsm_host.cpp: derive``)."""

    def __init__(self, cfg, dtype=np.float64):
        f = np.dtype(dtype).type
        self.dtype = np.dtype(dtype)
        self.N = int(cfg.n_agents)
        self.No = int(cfg.n_obstacles)
        self.E = 2 * self.N + self.No
        self.M = self.N + self.No
        self.L = f(np.float32(cfg.world_half)) if f is np.float32 else f(cfg.world_half)
        self.twoL = f(self.L * f(2))
        self.dt = f(cfg.dt)
        self.omd = f(f(1) - f(cfg.damping))
        self.mass = f(cfg.mass)
        self.cf = f(cfg.contact_force)
        self.k = f(cfg.contact_margin)
        self.sens = f(cfg.sensitivity)
        self.max_speed = f(cfg.max_speed)
        self.sa, self.sg, self.so = f(cfg.agent_size), f(cfg.goal_size), f(cfg.obstacle_size)
        self.R = f(cfg.sense_radius)
        self.R2 = f(self.R * self.R)
        # collider sizes in compact order: agents [0,N), obstacles [N, M)
        self.csize = np.concatenate([np.full(self.N, self.sa, self.dtype),
                                     np.full(self.No, self.so, self.dtype)])
        self.dmin = (self.sa + self.csize).astype(self.dtype)            # [M]
        self.dmin2 = (self.dmin * self.dmin).astype(self.dtype)          # [M]
        self.etype = np.concatenate([np.full(self.N, ENT_AGENT), np.full(self.N, ENT_GOAL),
                                     np.full(self.No, ENT_OBSTACLE)]).astype(np.int32)
        # compact collider index -> entity index
        self.cidx = np.concatenate([np.arange(self.N), 2 * self.N + np.arange(self.No)])


# ----------------------------------------------------------------------------
# reset: Philox layout (Appendix A S14 [DECISION]; replaces MPE np.random)
# ----------------------------------------------------------------------------
def layout(cfg, env_gids, episodes, seed=None):
    """Positions of every entity for (global env id, episode) pairs: fp32 [B,E,2].

    counter = (entity, episode, global env id, TAG_LAYOUT), key = (seed lo, hi);
    u = (x >> 8) * 2^-24;  p = u * (2L) - L   (two fp32 roundings, no FMA).
    """
    sp = Spec(cfg, np.float32)
    seed = int(cfg.seed if seed is None else seed)
    env_gids = np.asarray(env_gids, dtype=np.uint64)
    episodes = np.asarray(episodes, dtype=np.int64).astype(np.uint32)
    e = np.arange(sp.E, dtype=np.uint32)[None, :]
    x0, x1, _, _ = philox4x32_10(e, episodes[:, None], (env_gids & np.uint64(0xFFFFFFFF))[:, None],
                                 TAG_LAYOUT, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    L, twoL = np.float32(sp.L), np.float32(sp.twoL)
    px = u01_f32(x0) * twoL - L
    py = u01_f32(x1) * twoL - L
    return np.stack([px, py], axis=-1).astype(np.float32)


# ----------------------------------------------------------------------------
# Environment._set_action + World.apply_action_force (Appendix A S5)
# ----------------------------------------------------------------------------
def action_force(cfg, actions, fmt, dtype):
    """fmt 0: one-hot [B,N,5] -> u = [a1-a2, a3-a4]; fmt 1: index [B,N] (same
    mapping as the one-hot of that index; out-of-range = no-op); fmt 2:
    continuous [B,N,2]. Then u *= sensitivity (MPE: accel or 5.0)."""
    f = np.dtype(dtype).type
    sens = f(cfg.sensitivity)
    a = np.asarray(actions)
    if fmt == 0:
        a = a.astype(dtype)
        u = np.stack([a[..., 1] - a[..., 2], a[..., 3] - a[..., 4]], axis=-1)
    elif fmt == 1:
        k = a.astype(np.int64)
        ux = (k == 1).astype(dtype) - (k == 2).astype(dtype)
        uy = (k == 3).astype(dtype) - (k == 4).astype(dtype)
        u = np.stack([ux, uy], axis=-1)
    elif fmt == 2:
        u = a.astype(dtype)
    else:
        raise ValueError(fmt)
    return (u * sens).astype(dtype)


# ----------------------------------------------------------------------------
# World.step: apply_environment_force + integrate_state (Appendix A S3, S4, S6)
# ----------------------------------------------------------------------------
def physics(cfg, pos, vel, actions, fmt, dtype=np.float64):
    """One World.step for a batch. pos [B,E,2], vel [B,N,2] -> (pos', vel').

    Only agents are movable; goals (non-colliding) and obstacles (immovable)
    keep their positions. A coincident pair (d == 0) contributes zero force
    (Appendix A S16 guard), as does a pair with a non-finite distance. With
    ``cfg.strict_degenerate`` every pair is evaluated as MPE does: a coincident
    pair's force is 0/0 = NaN, and a NaN agent position makes every pair it
    is in NaN — hence every agent of its env, whose pair with it MPE always
    evaluates.
    """
    sp = Spec(cfg, dtype)
    f = sp.dtype.type
    N = sp.N
    pos = np.asarray(pos, dtype=dtype)
    vel = np.asarray(vel, dtype=dtype)
    pa = pos[:, :N]                                    # [B,N,2]
    pc = pos[:, sp.cidx]                               # [B,M,2]
    delta = pa[:, :, None, :] - pc[:, None, :, :]      # [B,N,M,2]
    dx, dy = delta[..., 0], delta[..., 1]
    d2 = dx * dx + dy * dy
    d = np.sqrt(d2)
    offdiag = ~np.eye(N, sp.M, dtype=bool)[None]
    strict = bool(getattr(cfg, "strict_degenerate", False))
    valid = offdiag if strict else (d2 > 0) & offdiag
    dsafe = np.where(valid, d, f(1))
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        pen = np.logaddexp(f(0), -(dsafe - sp.dmin[None, None, :]) / sp.k) * sp.k
        fx = np.where(valid, sp.cf * dx / dsafe * pen, f(0))
        fy = np.where(valid, sp.cf * dy / dsafe * pen, f(0))
    if strict:
        # a NaN agent j also reaches agent i through the pair (j, i) that MPE
        # evaluates from j's side; the [B,N,M] sum above covers (i, j) only
        bad_env = ~np.isfinite(pa).all(axis=(1, 2))
        fx[bad_env] = np.nan
        fy[bad_env] = np.nan
    F = action_force(cfg, actions, fmt, dtype) + np.stack([fx.sum(-1), fy.sum(-1)], axis=-1)
    v = vel * sp.omd
    with np.errstate(invalid="ignore"):
        v = v + (F / sp.mass) * sp.dt
    if sp.max_speed > 0:
        s = np.sqrt(v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1])
        over = s > sp.max_speed
        ssafe = np.where(over, s, f(1))
        v = np.where(over[..., None], v / ssafe[..., None] * sp.max_speed, v)
    new_pos = pos.copy()
    new_pos[:, :N] = pa + v * sp.dt
    return new_pos.astype(dtype), v.astype(dtype)


# ----------------------------------------------------------------------------
# scenario callbacks on the post-step state: reward, cost, graph observation
# ----------------------------------------------------------------------------
def _pair_d2(a, b):
    dx = a[..., 0] - b[..., 0]
    dy = a[..., 1] - b[..., 1]
    return dx * dx + dy * dy


def reward_cost(cfg, pos, dtype=np.float64):
    """reward [B,N] = -|p_i - g_i| (shared: sum over agents); cost [B,N] =
    number of agents/obstacles j != i in collision with agent i."""
    sp = Spec(cfg, dtype)
    N = sp.N
    pos = np.asarray(pos, dtype=dtype)
    pa, pg = pos[:, :N], pos[:, N:2 * N]
    r = -np.sqrt(_pair_d2(pa, pg))
    if cfg.shared_reward:
        r = np.repeat(r.sum(-1, keepdims=True), N, axis=-1)
    pc = pos[:, sp.cidx]
    d2 = _pair_d2(pa[:, :, None, :], pc[:, None, :, :])   # [B,N,M]
    if sp.dtype == np.float32:
        coll = d2 < sp.dmin2[None, None, :]
    else:
        coll = np.sqrt(d2) < sp.dmin[None, None, :]
    coll &= ~np.eye(N, sp.M, dtype=bool)[None]
    return r.astype(dtype), coll.sum(-1).astype(np.float32)


def node_features(cfg, pos, vel, dtype=np.float32):
    """node_feat [B,E,7]: [vx, vy, px, py, gx-px, gy-py, type] (goal-rel only for agents)."""
    sp = Spec(cfg, dtype)
    N = sp.N
    pos = np.asarray(pos, dtype=dtype)
    B = pos.shape[0]
    nf = np.zeros((B, sp.E, NODE_FEAT_DIM), dtype=dtype)
    nf[:, :N, 0:2] = vel
    nf[:, :, 2:4] = pos
    nf[:, :N, 4:6] = pos[:, N:2 * N] - pos[:, :N]
    nf[:, :, 6] = sp.etype.astype(dtype)
    return nf


def adjacency(cfg, pos, dtype=np.float64):
    """Dense directed connectivity [B,E,E] and pairwise d2 (Appendix A S8):
    radius edges among agents+obstacles (0 < d <= R, s != d) plus agent i <-> goal i."""
    sp = Spec(cfg, dtype)
    N = sp.N
    pos = np.asarray(pos, dtype=dtype)
    d2 = _pair_d2(pos[:, :, None, :], pos[:, None, :, :])        # [B,E,E]
    inAO = sp.etype != ENT_GOAL
    ao = inAO[:, None] & inAO[None, :]
    if sp.dtype == np.float32:
        rad = (d2 > 0) & (d2 <= sp.R2)
    else:
        dd = np.sqrt(d2)
        rad = (dd > 0) & (dd <= sp.R)
    conn = rad & ao[None]
    conn &= ~np.eye(sp.E, dtype=bool)[None]
    i = np.arange(N)
    conn[:, i, N + i] = True
    conn[:, N + i, i] = True
    return conn, d2


def edges(cfg, pos, dtype=np.float64):
    """Row-major COO over the batched graph (global node id = b*E + local).

    Returns edge_ptr [B+1] int64, edge_index [2, total] int32, edge_attr
    [total] (dist, in ``dtype``)."""
    sp = Spec(cfg, dtype)
    conn, d2 = adjacency(cfg, pos, dtype)
    B = conn.shape[0]
    b, s, t = np.nonzero(conn)                 # row-major (env, src, dst)
    counts = np.bincount(b, minlength=B)
    ptr = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(counts, out=ptr[1:])
    ei = np.stack([b * sp.E + s, b * sp.E + t]).astype(np.int32)
    attr = np.sqrt(d2[b, s, t]).astype(dtype)
    return ptr, ei, attr


# ----------------------------------------------------------------------------
# full step with episode bookkeeping and auto-reset (Appendix A S11)
# ----------------------------------------------------------------------------
def new_state(cfg, seed=None, dtype=np.float32):
    """State after reset(seed): episode index 0 for every env."""
    sp = Spec(cfg, dtype)
    B = int(cfg.n_envs)
    gids = int(cfg.env_base) + np.arange(B)
    return dict(
        pos=layout(cfg, gids, np.zeros(B, np.int64), seed).astype(dtype),
        vel=np.zeros((B, sp.N, 2), dtype=dtype),
        step=np.zeros(B, np.int32), episode=np.zeros(B, np.int32),
        ep_acc=np.zeros((B, 2), np.float64), ep_last=np.zeros((B, 2), np.float64),
    )


def degenerate(cfg, pos):
    """Appendix A S16 flags per env (uint8 [B]): 1 = two colliders, at least
    one an agent, at the same position (fp32 d2 = 0: the next step meets
    d = 0); 2 = an agent position is not finite."""
    sp = Spec(cfg, np.float32)
    N = sp.N
    pos = np.asarray(pos, dtype=np.float32)
    pa, pc = pos[:, :N], pos[:, sp.cidx]
    with np.errstate(invalid="ignore", over="ignore"):
        d2 = _pair_d2(pa[:, :, None, :], pc[:, None, :, :])       # [B,N,M] fp32
    coinc = ((d2 == 0) & ~np.eye(N, sp.M, dtype=bool)[None]).any(axis=(1, 2))
    nonfin = ~np.isfinite(pa).all(axis=(1, 2))
    return (coinc.astype(np.uint8) | (nonfin.astype(np.uint8) << 1)).astype(np.uint8)


def observe(cfg, st, dtype):
    pos, vel = st["pos"], st["vel"]
    r, c = reward_cost(cfg, pos, dtype)
    ptr, ei, attr = edges(cfg, pos, dtype)
    return dict(reward=r, cost=c, node_feat=node_features(cfg, pos, vel, dtype),
                edge_ptr=ptr, edge_index=ei, edge_attr=attr, degenerate=degenerate(cfg, pos))


def step(cfg, st, actions, fmt=1, dtype=np.float64, seed=None):
    """One env.step for the whole batch; returns (new_state, outputs).

    reward/cost are evaluated on the post-physics state; when an episode ends
    (t >= episode_length) and auto_reset is on, the env is re-laid-out
    (episode + 1) and node_feat/edges describe the reset state — the MAPPO
    vec-env convention (worker resets and returns the new obs on done).
    """
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    pos, vel = physics(cfg, st["pos"], st["vel"], actions, fmt, dtype)
    st["pos"], st["vel"] = pos, vel
    st["step"] = st["step"] + 1
    done = st["step"] >= int(cfg.episode_length)
    r, c = reward_cost(cfg, pos, dtype)
    st["ep_acc"] = st["ep_acc"] + np.stack([r.astype(np.float64).sum(-1),
                                            c.astype(np.float64).sum(-1)], -1)
    if cfg.auto_reset and done.any():
        idx = np.nonzero(done)[0]
        st["ep_last"][idx] = st["ep_acc"][idx]
        st["ep_acc"][idx] = 0
        st["episode"][idx] += 1
        gids = int(cfg.env_base) + idx
        st["pos"][idx] = layout(cfg, gids, st["episode"][idx], seed).astype(dtype)
        st["vel"][idx] = 0
        st["step"][idx] = 0
    ob = observe(cfg, st, dtype)
    ob["reward"], ob["cost"] = r, c
    ob["done"] = done.astype(np.uint8)
    return st, ob
