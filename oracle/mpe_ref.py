"""Object-per-entity restatement of the reference's MPE step path (fp64).

TEST INFRASTRUCTURE ONLY: the checker and the timed CPU baseline
(``bench.py`` ``cpu_baseline``, kind "port"). Never imported by the product.

This mirrors the *structure* of the hidden reference modules — entity objects,
a Python ``for a: for b > a`` contact loop, per-agent scenario callbacks — so
that timing it approximates what the reference's CPU ``World.step()`` costs
per env (SURVEY.md §3, §8(d) "CPU baseline"). The module paths it stands in
for are listed in ``/root/reference/GSMARL.egg-info/SOURCES.txt``:

* ``World``/``Entity``/``Agent``/``Landmark`` -> ``gsmarl/envs/mpe_env/multiagent/core.py`` (SOURCES.txt:14)
* ``GraphConstrainEnv.step/reset``            -> ``.../multiagent/environment.py`` (SOURCES.txt:15; readme.md:38-41)
* ``NavigationScenario``                      -> ``.../multiagent/scenarios/exp1.py`` / ``exp2.py`` (SOURCES.txt:21-22)

Their source is absent (readme.md:1), so the semantics are the upstream MPE
ones (readme.md:27 says the reference modifies MPE) + SURVEY.md Appendix A.
Parity with the true GS-MARL is unpinned (see ``oracle/batch_ref.py``).
"""
from __future__ import annotations

import numpy as np

from .batch_ref import ENT_AGENT, ENT_GOAL, ENT_OBSTACLE, layout, make_cfg


class EntityState:
    def __init__(self):
        self.p_pos = None
        self.p_vel = None


class Action:
    def __init__(self):
        self.u = None


class Entity:
    def __init__(self):
        self.name = ""
        self.size = 0.05
        self.movable = False
        self.collide = True
        self.initial_mass = 1.0
        self.max_speed = None
        self.accel = None
        self.state = EntityState()
        self.etype = ENT_OBSTACLE

    @property
    def mass(self):
        return self.initial_mass


class Landmark(Entity):
    pass


class Agent(Entity):
    def __init__(self):
        super().__init__()
        self.movable = True
        self.u_noise = None
        self.action = Action()
        self.etype = ENT_AGENT


class World:
    """MPE ``World`` with dim_p = 2, dim_c = 0 (Appendix A S1-S4, S6)."""

    def __init__(self):
        self.agents = []
        self.landmarks = []
        self.dim_p = 2
        self.dt = 0.1
        self.damping = 0.25
        self.contact_force = 1e2
        self.contact_margin = 1e-3
        self.strict = False   # Appendix A S16: True = MPE's unguarded 0/0 force

    @property
    def entities(self):
        return self.agents + self.landmarks

    def step(self):
        p_force = [None] * len(self.entities)
        p_force = self.apply_action_force(p_force)
        p_force = self.apply_environment_force(p_force)
        self.integrate_state(p_force)

    def apply_action_force(self, p_force):
        for i, agent in enumerate(self.agents):
            if agent.movable:
                p_force[i] = agent.action.u + 0.0
        return p_force

    def apply_environment_force(self, p_force):
        ents = self.entities
        for a, ea in enumerate(ents):
            for b in range(a + 1, len(ents)):
                f_a, f_b = self.get_collision_force(ea, ents[b])
                if f_a is not None:
                    p_force[a] = f_a + (0.0 if p_force[a] is None else p_force[a])
                if f_b is not None:
                    p_force[b] = f_b + (0.0 if p_force[b] is None else p_force[b])
        return p_force

    def get_collision_force(self, ea, eb):
        if not (ea.collide and eb.collide) or ea is eb:
            return None, None
        if not (ea.movable or eb.movable):
            return None, None
        delta = ea.state.p_pos - eb.state.p_pos
        dist = np.sqrt(np.sum(np.square(delta)))
        if not self.strict and not dist > 0.0:   # Appendix A S16 guard (MPE divides by 0)
            return None, None
        dist_min = ea.size + eb.size
        k = self.contact_margin
        with np.errstate(invalid="ignore", divide="ignore"):
            penetration = np.logaddexp(0, -(dist - dist_min) / k) * k
            force = self.contact_force * delta / dist * penetration
        return (+force if ea.movable else None), (-force if eb.movable else None)

    def integrate_state(self, p_force):
        for i, ent in enumerate(self.entities):
            if not ent.movable:
                continue
            ent.state.p_vel = ent.state.p_vel * (1 - self.damping)
            if p_force[i] is not None:
                ent.state.p_vel = ent.state.p_vel + (p_force[i] / ent.mass) * self.dt
            if ent.max_speed is not None:
                speed = np.sqrt(np.square(ent.state.p_vel[0]) + np.square(ent.state.p_vel[1]))
                if speed > ent.max_speed:
                    ent.state.p_vel = ent.state.p_vel / speed * ent.max_speed
            ent.state.p_pos = ent.state.p_pos + ent.state.p_vel * self.dt


class NavigationScenario:
    """Cooperative navigation: N agents, N goals (non-colliding), No obstacles."""

    def make_world(self, cfg):
        w = World()
        w.dt, w.damping = cfg.dt, cfg.damping
        w.contact_force, w.contact_margin = cfg.contact_force, cfg.contact_margin
        w.strict = bool(getattr(cfg, "strict_degenerate", False))
        self.cfg = cfg
        for i in range(cfg.n_agents):
            a = Agent()
            a.name, a.size, a.initial_mass = f"agent {i}", cfg.agent_size, cfg.mass
            a.accel = cfg.sensitivity
            a.max_speed = cfg.max_speed if cfg.max_speed > 0 else None
            w.agents.append(a)
        for i in range(cfg.n_agents):
            g = Landmark()
            g.name, g.size, g.collide, g.etype = f"goal {i}", cfg.goal_size, False, ENT_GOAL
            w.landmarks.append(g)
        for i in range(cfg.n_obstacles):
            o = Landmark()
            o.name, o.size, o.etype = f"obstacle {i}", cfg.obstacle_size, ENT_OBSTACLE
            w.landmarks.append(o)
        return w

    def reset_world(self, world, env_gid, episode, seed):
        pos = layout(self.cfg, [env_gid], [episode], seed)[0].astype(np.float64)
        for e, ent in enumerate(world.entities):
            ent.state.p_pos = pos[e].copy()
            ent.state.p_vel = np.zeros(world.dim_p)

    def goal(self, world, i):
        return world.landmarks[i]

    def reward(self, agent_idx, world):
        a = world.agents[agent_idx]
        return -float(np.sqrt(np.sum(np.square(a.state.p_pos - self.goal(world, agent_idx).state.p_pos))))

    @staticmethod
    def is_collision(e1, e2):
        delta = e1.state.p_pos - e2.state.p_pos
        return np.sqrt(np.sum(np.square(delta))) < e1.size + e2.size

    def cost(self, agent_idx, world):
        a = world.agents[agent_idx]
        n = 0
        for e in world.entities:
            if e is a or not e.collide:
                continue
            n += self.is_collision(a, e)
        return float(n)

    def observation(self, agent_idx, world):
        a = world.agents[agent_idx]
        g = self.goal(world, agent_idx)
        return np.concatenate([a.state.p_vel, a.state.p_pos, g.state.p_pos - a.state.p_pos])

    def node_table(self, world):
        rows = []
        n = len(world.agents)
        for e, ent in enumerate(world.entities):
            vel = ent.state.p_vel if ent.movable else np.zeros(2)
            grel = (world.landmarks[e].state.p_pos - ent.state.p_pos) if e < n else np.zeros(2)
            rows.append(np.concatenate([vel, ent.state.p_pos, grel, [float(ent.etype)]]))
        return np.array(rows)

    def graph(self, world):
        """Row-major edge list (src asc, dst asc) with distances (Appendix A S8)."""
        ents = world.entities
        n = len(world.agents)
        R = self.cfg.sense_radius
        src, dst, dist = [], [], []
        for s, es in enumerate(ents):
            for t, et in enumerate(ents):
                if s == t:
                    continue
                d = float(np.sqrt(np.sum(np.square(es.state.p_pos - et.state.p_pos))))
                goal_edge = (s < n and t == n + s) or (t < n and s == n + t)
                radius_edge = es.collide and et.collide and 0.0 < d <= R
                if goal_edge or radius_edge:
                    src.append(s)
                    dst.append(t)
                    dist.append(d)
        return np.array([src, dst], dtype=np.int64).reshape(2, -1), np.array(dist)


class GraphConstrainEnv:
    """Single-env MultiAgentGraphConstrainEnv restatement (readme.md:38-41)."""

    def __init__(self, cfg=None, env_gid=0, **kw):
        self.cfg = cfg if cfg is not None else make_cfg(**kw)
        self.scenario = NavigationScenario()
        self.world = self.scenario.make_world(self.cfg)
        self.n = self.cfg.n_agents
        self.env_gid = env_gid
        self.episode = -1
        self.current_step = 0

    def reset(self, seed=None):
        if seed is not None:
            self.cfg.seed = seed
            self.episode = -1
        self.episode += 1
        self.current_step = 0
        self.scenario.reset_world(self.world, self.env_gid, self.episode, self.cfg.seed)
        return self._obs()

    def _set_action(self, action, agent):
        """Discrete one-hot (MPE ``discrete_action_space``, not ``discrete_action_input``)."""
        agent.action.u = np.zeros(self.world.dim_p)
        agent.action.u[0] += action[1] - action[2]
        agent.action.u[1] += action[3] - action[4]
        agent.action.u *= agent.accel if agent.accel is not None else 5.0

    def _obs(self):
        obs_n = [self.scenario.observation(i, self.world) for i in range(self.n)]
        ei, dist = self.scenario.graph(self.world)
        return obs_n, self.scenario.node_table(self.world), ei, dist

    def step(self, action_n):
        for i, agent in enumerate(self.world.agents):
            self._set_action(np.asarray(action_n[i], dtype=np.float64), agent)
        self.world.step()
        self.current_step += 1
        reward_n = [self.scenario.reward(i, self.world) for i in range(self.n)]
        if self.cfg.shared_reward:
            reward_n = [float(np.sum(reward_n))] * self.n
        cost_n = [self.scenario.cost(i, self.world) for i in range(self.n)]
        done = self.current_step >= self.cfg.episode_length
        done_n = [done] * self.n
        info_n = [{"cost": c} for c in cost_n]
        obs_n, node, ei, dist = self._obs()
        return obs_n, node, ei, dist, reward_n, cost_n, done_n, info_n

    # state injection for parity tests (SURVEY.md §5 checkpoint/resume)
    def set_state(self, pos, vel):
        for e, ent in enumerate(self.world.entities):
            ent.state.p_pos = np.array(pos[e], dtype=np.float64)
            ent.state.p_vel = np.array(vel[e], dtype=np.float64) if e < self.n else np.zeros(2)

    def get_state(self):
        pos = np.array([e.state.p_pos for e in self.world.entities])
        vel = np.array([a.state.p_vel for a in self.world.agents])
        return pos, vel
