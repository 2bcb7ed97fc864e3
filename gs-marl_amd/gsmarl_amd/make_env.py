"""Env factory — stands in for ``gsmarl/envs/mpe_env/make_env.py``
(SOURCES.txt:12): scenario name + parameters -> env object."""
from __future__ import annotations

from .config import EnvConfig
from .environment import MultiAgentConstrainEnv, MultiAgentEnv, MultiAgentGraphConstrainEnv

ENV_CLASSES = {
    "MultiAgentEnv": MultiAgentEnv,
    "MultiAgentConstrainEnv": MultiAgentConstrainEnv,
    "MultiAgentGraphConstrainEnv": MultiAgentGraphConstrainEnv,
}


# the reference's scenario module names (SOURCES.txt:21-25) -> scenario
SCENARIO_ALIASES = {
    "exp1": "navigation", "exp2": "navigation", "navigation": "navigation",
    "simple_formation": "polygon", "formation": "polygon", "polygon": "polygon",
    "simple_line": "line", "line": "line", "mixed": "mixed",
}


def make_env(scenario_name: str = "navigation", env_class: str = "MultiAgentGraphConstrainEnv",
             device="cuda", **params):
    try:
        scenario = SCENARIO_ALIASES[scenario_name]
    except KeyError:
        raise ValueError(f"unknown scenario {scenario_name!r}; have {sorted(SCENARIO_ALIASES)}") from None
    cfg = EnvConfig(scenario=scenario, **params)
    try:
        cls = ENV_CLASSES[env_class]
    except KeyError:
        raise ValueError(f"unknown env class {env_class!r}; have {sorted(ENV_CLASSES)}") from None
    return cls(cfg, device=device)
