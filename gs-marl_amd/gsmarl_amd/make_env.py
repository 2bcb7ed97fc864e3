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


def make_env(scenario_name: str = "navigation", env_class: str = "MultiAgentGraphConstrainEnv",
             device="cuda", **params):
    cfg = EnvConfig(scenario=scenario_name, **params)
    try:
        cls = ENV_CLASSES[env_class]
    except KeyError:
        raise ValueError(f"unknown env class {env_class!r}; have {sorted(ENV_CLASSES)}") from None
    return cls(cfg, device=device)
