"""ctypes binding of libgsm.so (the C ABI in include/gsm.h).

The library is built in-tree by ``__graft_entry__.build()`` into
``gs-marl_amd/gsmarl_amd/lib/libgsm.so``. There is no fallback: if it is
missing, or no GPU is visible, the product path raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("GSM_LIB_PATH") or Path(__file__).resolve().parent / "lib" / "libgsm.so")
ABI_VERSION = 8
DEGENERATE_COINCIDENT, DEGENERATE_NONFINITE = 1, 2

GSM_OK, GSM_EINVAL, GSM_EHIP, GSM_ESTATE = 0, -1, -2, -3
GRAPH_SLOTS = 4
GRAPH_STEP, GRAPH_EMIT, GRAPH_TIME_EACH, GRAPH_TIME_ENDS = 1, 2, 4, 8
GRAPH_UNFUSED, GRAPH_LAG_ONLY, GRAPH_ROLL = 16, 32, 64
RENDER_EDGES = 1
ACT_ONEHOT, ACT_INDEX, ACT_CONT = 0, 1, 2


class GsmConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("scenario", C.c_int32), ("n_envs", C.c_int32),
        ("n_agents", C.c_int32), ("n_obstacles", C.c_int32), ("episode_length", C.c_int32),
        ("auto_reset", C.c_int32), ("shared_reward", C.c_int32),
        ("env_base", C.c_int64), ("seed", C.c_uint64),
        ("dt", C.c_float), ("damping", C.c_float), ("mass", C.c_float),
        ("contact_force", C.c_float), ("contact_margin", C.c_float), ("sensitivity", C.c_float),
        ("max_speed", C.c_float), ("world_half", C.c_float),
        ("agent_size", C.c_float), ("goal_size", C.c_float), ("obstacle_size", C.c_float),
        ("sense_radius", C.c_float), ("contact_cutoff", C.c_float),
        ("n_agents_min", C.c_int32), ("formation_radius", C.c_float),
        ("strict_degenerate", C.c_int32),
    ]


class GsmSizes(C.Structure):
    _fields_ = [
        ("n_entities", C.c_int32), ("node_feat_dim", C.c_int32), ("obs_dim", C.c_int32),
        ("envs_per_block", C.c_int32), ("n_blocks", C.c_int32), ("max_edges_per_env", C.c_int32),
        ("edge_capacity", C.c_int64), ("n_colliders", C.c_int32), ("n_targets", C.c_int32),
        ("mask_words", C.c_int32),
    ]


BUFFER_FIELDS = ["pos", "vel", "step_count", "episode", "ep_acc", "ep_last", "node_feat",
                 "reward", "cost", "done", "edge_count", "block_edge_sum", "edge_ptr",
                 "edge_index", "edge_attr", "row_mask", "contact_mask", "env_shape", "assign", "degenerate",
                 "lsa_v", "lsa_col", "lsa_stats"]


class GsmBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in BUFFER_FIELDS]


OUTPUT_FIELDS = ["node_feat", "reward", "cost", "done", "edge_count", "edge_ptr", "edge_index", "edge_attr",
                 "assign"]


class GsmOutputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in OUTPUT_FIELDS] + [("edge_capacity", C.c_int64)]


STATE_FIELDS = ["pos", "vel", "step_count", "episode", "ep_acc", "ep_last", "env_shape"]


class GsmState(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in STATE_FIELDS]


# every symbol include/gsm.h declares, with its ctypes signature
_P = C.c_void_p
SIGNATURES = {
    "gsm_abi_version": (C.c_int, []),
    "gsm_query_sizes": (C.c_int, [C.POINTER(GsmConfig), C.POINTER(GsmSizes)]),
    "gsm_create": (C.c_int, [C.POINTER(GsmConfig), C.POINTER(_P)]),
    "gsm_bind": (C.c_int, [_P, C.POINTER(GsmBuffers)]),
    "gsm_reset": (C.c_int, [_P, C.c_uint64, C.c_int, _P, _P]),
    "gsm_step": (C.c_int, [_P, _P, C.c_int, _P]),
    "gsm_observe": (C.c_int, [_P, _P]),
    "gsm_get_state": (C.c_int, [_P, C.POINTER(GsmState), _P]),
    "gsm_set_state": (C.c_int, [_P, C.POINTER(GsmState), _P]),
    "gsm_step_into": (C.c_int, [_P, _P, C.c_int, C.POINTER(GsmOutputs), _P]),
    "gsm_observe_into": (C.c_int, [_P, C.POINTER(GsmOutputs), _P]),
    "gsm_graph_capture_into": (C.c_int, [_P, C.c_int32, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int,
                                         C.POINTER(GsmOutputs)]),
    "gsm_graph_capture": (C.c_int, [_P, C.c_int32, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int, C.c_int]),
    "gsm_graph_launch": (C.c_int, [_P, C.c_int32, _P]),
    "gsm_graph_roll_status": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "gsm_graph_roll_placement": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "gsm_graph_info": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "gsm_graph_kernel_ms": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                      C.POINTER(C.c_float)]),
    "gsm_attn_aggregate": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_float,
                                     _P, _P]),
    "gsm_render": (C.c_int, [_P, C.c_int64, C.c_int32, _P, _P, C.c_int64, _P, C.c_int32, C.c_float, C.c_float,
                             C.c_float, C.c_float, C.c_int32, C.c_int32, C.c_int32, _P, _P]),
    "gsm_debug_set_stamps": (C.c_int, [_P, _P]),
    "gsm_destroy": (C.c_int, [_P]),
    "gsm_last_error": (C.c_int, [_P, C.c_char_p, C.c_size_t]),
}

_lib = None


class GsmError(RuntimeError):
    pass


def load(path: os.PathLike | None = None):
    """Load (once) and type the library. Raises if it has not been built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise GsmError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gsm_abi_version() != ABI_VERSION:
        raise GsmError(f"libgsm ABI {lib.gsm_abi_version()} != binding ABI {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def last_error(lib, handle=None) -> str:
    buf = C.create_string_buffer(1024)
    lib.gsm_last_error(handle, buf, len(buf))
    return buf.value.decode(errors="replace")


def check(lib, rc: int, handle=None, what: str = "") -> None:
    if rc != GSM_OK:
        raise GsmError(f"{what} failed (status {rc}): {last_error(lib, handle)}")


def make_config(cfg) -> GsmConfig:
    from .config import SCENARIOS
    c = GsmConfig()
    c.abi_version = ABI_VERSION
    c.scenario = SCENARIOS[cfg.scenario]
    c.n_envs, c.n_agents, c.n_obstacles = int(cfg.n_envs), int(cfg.n_agents), int(cfg.n_obstacles)
    c.episode_length = int(cfg.episode_length)
    c.auto_reset, c.shared_reward = int(bool(cfg.auto_reset)), int(bool(cfg.shared_reward))
    c.env_base, c.seed = int(cfg.env_base), int(cfg.seed) & 0xFFFFFFFFFFFFFFFF
    for f in ("dt", "damping", "mass", "contact_force", "contact_margin", "sensitivity",
              "max_speed", "world_half", "agent_size", "goal_size", "obstacle_size",
              "sense_radius", "contact_cutoff", "formation_radius"):
        setattr(c, f, float(getattr(cfg, f)))
    c.n_agents_min = int(cfg.n_agents_min)
    c.strict_degenerate = int(bool(getattr(cfg, "strict_degenerate", False)))
    return c


def query_sizes(cfg, lib=None) -> GsmSizes:
    lib = lib or load()
    c = make_config(cfg)
    s = GsmSizes()
    check(lib, lib.gsm_query_sizes(C.byref(c), C.byref(s)), None, "gsm_query_sizes")
    return s
