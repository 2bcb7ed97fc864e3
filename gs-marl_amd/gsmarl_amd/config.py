"""Env configuration — the env-relevant subset of the reference's
``gsmarl/config.py`` (SOURCES.txt:7, readme.md:47) plus the MPE constants of
``core.py`` / the scenario files, mirrored 1:1 into ``gsm_config``
(include/gsm.h). Defaults are SURVEY.md Appendix A (S2, S3, S5, S10, S11)."""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field, replace
from typing import Optional

SCENARIOS = {"navigation": 0, "polygon": 1, "line": 2, "mixed": 3}
RAGGED_MAX_AGENTS = 32   # gsm.h GSM_RAGGED_MAX_AGENTS


@dataclass
class EnvConfig:
    scenario: str = "navigation"
    n_envs: int = 1
    n_agents: int = 3
    n_obstacles: Optional[int] = None      # default: n_agents (navigation, mixed), 0 (polygon, line)
    episode_length: int = 100              # readme.md:101
    auto_reset: bool = True
    shared_reward: bool = False
    env_base: int = 0                      # global id of env 0 (sharding)
    seed: int = 0
    dt: float = 0.1
    damping: float = 0.25
    mass: float = 1.0
    contact_force: float = 100.0
    contact_margin: float = 1e-3
    sensitivity: float = 5.0               # MPE: accel or 5.0
    max_speed: float = 0.0                 # <= 0: None
    world_half: Optional[float] = None     # default sqrt(N/3); polygon/line/mixed: 0 = per env sqrt(N_env/3)
    agent_size: float = 0.05
    goal_size: float = 0.05
    obstacle_size: float = 0.08
    sense_radius: float = 0.5
    contact_cutoff: float = 40.0           # in contact margins
    n_agents_min: int = 3                  # mixed: N_env drawn from [n_agents_min, n_agents]
    formation_radius: float = 0.5          # polygon N-gon radius (readme.md:89)
    strict_degenerate: bool = False        # App. A S16: MPE's NaN for d = 0 pairs instead of the guard
    lsa_warm_start: bool = True            # polygon/line: certified warm-started assignment (gsm.h lsa_v)

    def __post_init__(self):
        if self.scenario not in SCENARIOS:
            raise ValueError(f"unknown scenario {self.scenario!r}; have {sorted(SCENARIOS)}")
        if self.n_obstacles is None:
            self.n_obstacles = self.n_agents if self.scenario in ("navigation", "mixed") else 0
        if self.world_half is None:
            self.world_half = math.sqrt(self.n_agents / 3.0) if not self.ragged else 0.0
        self.n_agents_min = min(self.n_agents_min, self.n_agents)

    @property
    def ragged(self) -> bool:
        """Polygon, line and mixed batches: per-env N_env <= n_agents, padded."""
        return self.scenario != "navigation"

    @property
    def n_targets(self) -> int:
        return {"polygon": 1, "line": 2}.get(self.scenario, self.n_agents)

    @property
    def n_entities(self) -> int:
        return self.n_agents + self.n_targets + self.n_obstacles

    def replace(self, **kw) -> "EnvConfig":
        return replace(self, **kw)

    def to_dict(self) -> dict:
        return asdict(self)
