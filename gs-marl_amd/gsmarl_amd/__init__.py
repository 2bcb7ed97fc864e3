"""gsmarl_amd — MI355X-native batched step path of GS-MARL's
MultiAgentGraphConstrainEnv (HIP kernels in libgsm.so behind a C ABI)."""
from .config import EnvConfig
from .batch import GpuBatchEnv
from .environment import MultiAgentConstrainEnv, MultiAgentEnv, MultiAgentGraphConstrainEnv
from .make_env import make_env
from .vec_env import GpuGraphVecEnv, make_eval_env, make_train_env
from .rollout import GraphRolloutBuffer
from . import gnn
from . import render
from . import distributed

__version__ = "0.1.0"
__all__ = ["EnvConfig", "GpuBatchEnv", "MultiAgentEnv", "MultiAgentConstrainEnv",
           "MultiAgentGraphConstrainEnv", "make_env", "GpuGraphVecEnv", "make_train_env", "make_eval_env",
           "GraphRolloutBuffer", "gnn", "render",
           "distributed"]
