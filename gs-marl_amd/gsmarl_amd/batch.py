"""GpuBatchEnv — B independent MultiAgentGraphConstrainEnv instances resident
in HBM, stepped by the HIP kernels in libgsm.so.

State and outputs are PyTorch device tensors (PyTorch is the allocator and
stream provider only); every compute call goes through the C ABI. Layout
(SoA over envs):

    pos        [B, E, 2] f32   agents [0,N), goals [N,2N), obstacles [2N,E)
    vel        [B, N, 2] f32
    node_feat  [B, E, 7] f32   vx vy px py gx-px gy-py type
    obs        [B, N, 6]       = node_feat[:, :N, :6]  (a view: MPE obs order)
    reward     [B, N] f32, cost [B, N] f32 (exact counts), done [B] u8
    degenerate [B] u8      App. A S16 flags: 1 coincident collider pair, 2 non-finite agent
    edge_ptr   [B+1] i64; edge_index [2, cap] i32 (global node ids b*E+e),
    edge_attr  [cap] f32 (distance); valid prefix = edge_ptr[B]
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

from . import _lib
from .config import EnvConfig

# roctx ranges around every launch call (GSM_ROCTX=1; torch.cuda.nvtx is
# roctx on ROCm), so rocprofv3 --marker-trace timelines show env.step /
# reset / observe / graph replays next to their kernels. Off by default.
_ROCTX = os.environ.get("GSM_ROCTX", "") not in ("", "0")


def _ranged(name):
    def deco(fn):
        if not _ROCTX:
            return fn

        def wrapped(*a, **kw):
            torch.cuda.nvtx.range_push(name)
            try:
                return fn(*a, **kw)
            finally:
                torch.cuda.nvtx.range_pop()
        wrapped.__name__, wrapped.__doc__ = fn.__name__, fn.__doc__
        return wrapped
    return deco


def _require_gpu(device) -> torch.device:
    device = torch.device(device)
    if device.type != "cuda" or not torch.cuda.is_available():
        raise _lib.GsmError("GpuBatchEnv needs a ROCm GPU (torch.cuda.is_available() is False); "
                            "there is no CPU fallback by design")
    return device


class GpuBatchEnv:
    """Batched navigation env; ``step``/``reset`` are asynchronous on the
    current torch stream and return dicts of device tensors."""

    def __init__(self, cfg: EnvConfig, device="cuda"):
        self.cfg = cfg
        self.device = _require_gpu(device)
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.lib = _lib.load()
        self._launch = self.lib.gsm_graph_launch
        self.sizes = _lib.query_sizes(cfg, self.lib)
        self._ccfg = _lib.make_config(cfg)
        h = C.c_void_p()
        _lib.check(self.lib, self.lib.gsm_create(C.byref(self._ccfg), C.byref(h)), None, "gsm_create")
        self._h = h
        B, N, E = cfg.n_envs, cfg.n_agents, self.sizes.n_entities
        self.B, self.N, self.E = B, N, E
        dev = self.device
        f32, i32 = torch.float32, torch.int32
        cap = int(self.sizes.edge_capacity)
        self.t = dict(
            pos=torch.zeros(B, E, 2, dtype=f32, device=dev),
            vel=torch.zeros(B, N, 2, dtype=f32, device=dev),
            step_count=torch.zeros(B, dtype=i32, device=dev),
            episode=torch.full((B,), -1, dtype=i32, device=dev),
            ep_acc=torch.zeros(B, 2, dtype=f32, device=dev),
            ep_last=torch.zeros(B, 2, dtype=f32, device=dev),
            node_feat=torch.zeros(B, E, 7, dtype=f32, device=dev),
            reward=torch.zeros(B, N, dtype=f32, device=dev),
            cost=torch.zeros(B, N, dtype=f32, device=dev),
            done=torch.zeros(B, dtype=torch.uint8, device=dev),
            edge_count=torch.zeros(B, dtype=i32, device=dev),
            block_edge_sum=torch.zeros(self.sizes.n_blocks, dtype=i32, device=dev),
            edge_ptr=torch.zeros(B + 1, dtype=torch.int64, device=dev),
            edge_index=torch.zeros(2, cap, dtype=i32, device=dev),
            edge_attr=torch.zeros(cap, dtype=f32, device=dev),
            # derived state (refreshed by every reset/step/observe)
            row_mask=torch.zeros(B, self.sizes.n_colliders * self.sizes.mask_words, dtype=torch.int64,
                                 device=dev),
            contact_mask=torch.zeros(B, N * self.sizes.mask_words, dtype=torch.int64, device=dev),
            # ragged batches: N_env | scenario << 8, and the LSA slot of each agent
            env_shape=torch.zeros(B, dtype=i32, device=dev),
            assign=torch.full((B, N), -1, dtype=i32, device=dev),
            # App. A S16 flags per env (GSM_DEGENERATE_*: 1 coincident pair, 2 non-finite agent)
            degenerate=torch.zeros(B, dtype=torch.uint8, device=dev),
            # ragged assignment warm start (column duals, matching) and its counters
            lsa_v=torch.zeros(B, N, dtype=torch.float64, device=dev),
            lsa_col=torch.full((B, N), -1, dtype=i32, device=dev),
            lsa_stats=torch.zeros(B, 2, dtype=i32, device=dev),
        )
        ptrs = {k: self.t[k].data_ptr() for k in _lib.BUFFER_FIELDS}
        if not cfg.lsa_warm_start:   # every assignment solved from scratch
            ptrs["lsa_v"] = ptrs["lsa_col"] = None
        bufs = _lib.GsmBuffers(**ptrs)
        _lib.check(self.lib, self.lib.gsm_bind(self._h, C.byref(bufs)), self._h, "gsm_bind")
        self.agent_id = torch.arange(N, dtype=torch.int64, device=dev).expand(B, N)
        self._graph_actions = {}

    # ------------------------------------------------------------------ utils
    def _stream(self):
        # the raw handle of the current stream (torch's own accessor: no
        # Stream object built per call)
        return C.c_void_p(torch._C._cuda_getCurrentRawStream(self._dev_index))

    def _chk(self, rc, what):
        _lib.check(self.lib, rc, self._h, what)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.gsm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------- outputs
    def outputs(self, sync_edges: bool = True) -> dict:
        t = self.t
        out = dict(obs=t["node_feat"][:, : self.N, :6], node_feat=t["node_feat"],
                   agent_id=self.agent_id, reward=t["reward"], cost=t["cost"], done=t["done"],
                   edge_ptr=t["edge_ptr"], degenerate=t["degenerate"])
        if self.cfg.ragged:
            out["assign"] = t["assign"]
            out["n_agents_env"] = t["env_shape"] & 0xFF
            out["scenario_env"] = t["env_shape"] >> 8
        if sync_edges:
            total = int(t["edge_ptr"][self.B].item())
            out["edge_index"] = t["edge_index"][:, :total]
            out["edge_attr"] = t["edge_attr"][:total]
        else:
            out["edge_index"] = t["edge_index"]
            out["edge_attr"] = t["edge_attr"]
        return out

    # ------------------------------------------------------------------- API
    @_ranged("gsm.reset")
    def reset(self, seed: Optional[int] = None, env_mask: Optional[torch.Tensor] = None,
              sync_edges: bool = True) -> dict:
        """Re-lay-out the masked envs (all if None). With ``seed`` the episode
        counters restart and ``seed`` keys every later layout."""
        mask_ptr = None
        if env_mask is not None:
            env_mask = env_mask.to(device=self.device, dtype=torch.uint8).contiguous()
            if env_mask.numel() != self.B:
                raise ValueError("env_mask must have n_envs elements")
            mask_ptr = C.c_void_p(env_mask.data_ptr())
        reseed = seed is not None
        if reseed:
            self.cfg.seed = int(seed)
        s = int(seed) & 0xFFFFFFFFFFFFFFFF if reseed else 0
        self._chk(self.lib.gsm_reset(self._h, s, int(reseed), mask_ptr, self._stream()), "gsm_reset")
        return self.outputs(sync_edges)

    def _action_fmt(self, actions: torch.Tensor) -> int:
        B, N = self.B, self.N
        if actions.device != self.device:
            raise ValueError("actions must be on the env's device")
        if actions.dtype == torch.int32 and tuple(actions.shape) == (B, N):
            return _lib.ACT_INDEX
        if actions.dtype == torch.float32 and tuple(actions.shape) == (B, N, 5):
            return _lib.ACT_ONEHOT
        if actions.dtype == torch.float32 and tuple(actions.shape) == (B, N, 2):
            return _lib.ACT_CONT
        raise ValueError(f"actions must be int32 [B,N], float32 one-hot [B,N,5] or float32 [B,N,2]; "
                         f"got {actions.dtype} {tuple(actions.shape)}")

    def _outputs_struct(self, out: dict) -> "_lib.GsmOutputs":
        """gsm_outputs for a dict of device tensors (missing keys keep the
        bound buffers). Shapes must match the bound outputs; edge arrays may be
        smaller than the worst case (edge_index [2, cap], edge_attr [cap])."""
        o = _lib.GsmOutputs()
        for k, v in out.items():
            if k not in _lib.OUTPUT_FIELDS:
                raise KeyError(f"not a redirectable output: {k}")
            ref = self.t[k]
            if v.device != self.device or v.dtype != ref.dtype or not v.is_contiguous():
                raise ValueError(f"output {k}: need a contiguous {ref.dtype} tensor on {self.device}")
            if k in ("edge_index", "edge_attr"):
                continue
            if v.shape != ref.shape:
                raise ValueError(f"output {k}: shape {tuple(v.shape)} != {tuple(ref.shape)}")
            setattr(o, k, v.data_ptr())
        if ("edge_index" in out) != ("edge_attr" in out):
            raise ValueError("edge_index and edge_attr are redirected together")
        if "edge_index" in out:
            ei, ea = out["edge_index"], out["edge_attr"]
            if ei.dim() != 2 or ei.shape[0] != 2 or ea.shape != (ei.shape[1],):
                raise ValueError("edge_index must be [2, cap] and edge_attr [cap]")
            o.edge_index, o.edge_attr, o.edge_capacity = ei.data_ptr(), ea.data_ptr(), int(ei.shape[1])
        return o

    @_ranged("gsm.step")
    def step(self, actions: torch.Tensor, sync_edges: bool = True, out: Optional[dict] = None) -> dict:
        """One env.step. With ``out`` (a dict of device tensors, e.g. a rollout
        buffer slot) the step writes those outputs there instead (no copies)."""
        if not actions.is_contiguous():
            actions = actions.contiguous()
        fmt = self._action_fmt(actions)
        a = C.c_void_p(actions.data_ptr())
        if out is None:
            self._chk(self.lib.gsm_step(self._h, a, fmt, self._stream()), "gsm_step")
            return self.outputs(sync_edges)
        o = self._outputs_struct(out)
        self._chk(self.lib.gsm_step_into(self._h, a, fmt, C.byref(o), self._stream()), "gsm_step_into")
        return out

    @_ranged("gsm.observe")
    def observe(self, sync_edges: bool = True, out: Optional[dict] = None) -> dict:
        if out is None:
            self._chk(self.lib.gsm_observe(self._h, self._stream()), "gsm_observe")
            return self.outputs(sync_edges)
        o = self._outputs_struct(out)
        self._chk(self.lib.gsm_observe_into(self._h, C.byref(o), self._stream()), "gsm_observe_into")
        return out

    # ------------------------------------------------- checkpoint / injection
    STATE_KEYS = ("pos", "vel", "step_count", "episode", "ep_acc", "ep_last")

    def render(self, env_ids=(0,), width: int = 700, height: int = 700, edges: bool = True) -> torch.Tensor:
        """RGB frames uint8 [n, H, W, 3] of the current state of envs
        ``env_ids`` (gsmarl_amd.render; camera [-L, L]^2 of each env)."""
        from .render import render_frames
        c = self.cfg
        return render_frames(self.t["node_feat"], self.t["edge_ptr"], self.t["edge_index"], env_ids, width, height,
                             (c.agent_size, c.goal_size, c.obstacle_size), c.world_half or 0.0, edges)

    def _state_keys(self):
        return self.STATE_KEYS + (("env_shape",) if self.cfg.ragged else ())

    def get_state(self) -> dict:
        """A copy of the simulator state (gsm_get_state): pos, vel, step_count,
        episode, ep_acc, ep_last (+ env_shape for ragged batches)."""
        out = {k: torch.empty_like(self.t[k]) for k in self._state_keys()}
        st = _lib.GsmState(**{k: v.data_ptr() for k, v in out.items()})
        self._chk(self.lib.gsm_get_state(self._h, C.byref(st), self._stream()), "gsm_get_state")
        return out

    def set_state(self, state: dict, sync_edges: bool = True) -> dict:
        """Overwrite state buffers and re-observe (gsm_set_state: the observe
        also refreshes the derived per-position state the next step relies on).
        Missing keys keep their current values."""
        src = {}
        for k, v in state.items():
            if k not in self._state_keys():
                raise KeyError(k)
            t = torch.as_tensor(v).to(device=self.device, dtype=self.t[k].dtype).contiguous()
            if t.shape != self.t[k].shape:
                raise ValueError(f"state {k}: shape {tuple(t.shape)} != {tuple(self.t[k].shape)}")
            src[k] = t
        st = _lib.GsmState(**{k: v.data_ptr() for k, v in src.items()})
        self._chk(self.lib.gsm_set_state(self._h, C.byref(st), self._stream()), "gsm_set_state")
        self._state_src = src   # keep the sources alive until the stream has copied them
        return self.outputs(sync_edges)

    # ------------------------------------------------------------ HIP graph
    def capture(self, actions_seq: Optional[torch.Tensor], n_steps: int, timing: bool = False,
                slot: int = 0, kernels: str = "both", time_ends: bool = False) -> None:
        """Build HIP graph ``slot`` of ``n_steps`` steps; the j-th step uses
        ``actions_seq[j % len(actions_seq)]`` (a [T, B, N(,k)] device tensor).
        kernels: "both" (segmented configs: lagged emission, one launch per
        step), "unfused" (step + emit kernel per step), "step", "emit"
        (re-emits the current edges), "lag" (lagged step kernels only; the
        last step's edges are left unemitted — a timing tool) or "roll"
        (all n_steps steps and their edges in ONE fused rollout launch;
        navigation configs with a compiled rollout shape (3, 6, 12 or 24
        agents with as many obstacles) or the tile path — GsmError otherwise;
        with time_ends the events bracket that launch).
        timing: event nodes around every kernel (implies "unfused");
        time_ends: only around the whole graph (per-kernel means over
        back-to-back launches)."""
        flags = {"both": 0, "unfused": _lib.GRAPH_UNFUSED, "step": _lib.GRAPH_STEP, "emit": _lib.GRAPH_EMIT,
                 "lag": _lib.GRAPH_LAG_ONLY, "roll": _lib.GRAPH_ROLL}[kernels]
        if timing:
            flags |= _lib.GRAPH_TIME_EACH
        if time_ends:
            flags |= _lib.GRAPH_TIME_ENDS
        if actions_seq is None:
            a, fmt, stride, n_act, ptr = None, _lib.ACT_INDEX, 0, 1, None
        else:
            a = actions_seq.contiguous()
            fmt = self._action_fmt(a[0])
            stride = a[0].numel() * a.element_size()
            n_act, ptr = a.shape[0], C.c_void_p(a.data_ptr())
        self._graph_actions[slot] = a   # keep alive while the graph exists
        self._chk(self.lib.gsm_graph_capture(self._h, int(slot), ptr, stride, n_act, int(n_steps), fmt,
                                             flags), "gsm_graph_capture")

    def capture_into(self, actions_seq: torch.Tensor, outs: list, slot: int = 0) -> None:
        """HIP graph of len(outs) steps; the j-th step uses actions_seq[j %
        len(actions_seq)] and writes its outputs to outs[j] (dicts as in step)."""
        a = actions_seq.contiguous()
        fmt = self._action_fmt(a[0])
        stride = a[0].numel() * a.element_size()
        arr = (_lib.GsmOutputs * len(outs))(*[self._outputs_struct(o) for o in outs])
        self._graph_actions[slot] = (a, outs)   # keep alive while the graph exists
        self._chk(self.lib.gsm_graph_capture_into(self._h, int(slot), C.c_void_p(a.data_ptr()), stride,
                                                  a.shape[0], len(outs), fmt, arr), "gsm_graph_capture_into")

    @_ranged("gsm.replay")
    def replay(self, slot: int = 0) -> None:
        # (the hot path of a training loop: one C call, the error path only
        # on a non-zero return)
        rc = self._launch(self._h, slot, torch._C._cuda_getCurrentRawStream(self._dev_index))
        if rc:
            self._chk(rc, "gsm_graph_launch")

    def graph_is_rollout(self, slot: int = 0) -> bool:
        """Whether graph ``slot`` is one fused rollout launch (GSM_GRAPH_ROLL,
        or capture_into on a rollout buffer) rather than a per-step chain."""
        steps, fused = C.c_int32(), C.c_int32()
        self._chk(self.lib.gsm_graph_info(self._h, int(slot), C.byref(steps), C.byref(fused)), "gsm_graph_info")
        return bool(fused.value)

    def roll_gave_up(self) -> int:
        """Whether a bounded in-launch wait (a fused rollout launch, or the
        ragged lagged chain's staging wait) timed out since the last call
        (outputs of that launch invalid); clears the flag. Synchronises."""
        v = C.c_int32()
        self._chk(self.lib.gsm_graph_roll_status(self._h, C.byref(v)), "gsm_graph_roll_status")
        return v.value   # truthy: the reason code (gsm.h gsm_graph_roll_status)

    def roll_placement(self) -> tuple:
        """(dealt, fell_back): ragged mixed rollout launches since the last
        call that dealt their envs to the SIMDs by cost, and that ran env =
        wave index because not every wave was resident (gsm.h
        gsm_graph_roll_placement); clears the counts. Synchronises."""
        d, f = C.c_int64(), C.c_int64()
        self._chk(self.lib.gsm_graph_roll_placement(self._h, C.byref(d), C.byref(f)), "gsm_graph_roll_placement")
        return int(d.value), int(f.value)

    def graph_kernel_ms(self, slot: int = 0):
        """(mean step-kernel ms, mean emit-kernel ms, whole-graph ms) of the
        last replay of a timed graph."""
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        self._chk(self.lib.gsm_graph_kernel_ms(self._h, int(slot), C.byref(a), C.byref(b), C.byref(c)),
                  "gsm_graph_kernel_ms")
        return a.value, b.value, c.value

    def lsa_warm_stats(self) -> tuple:
        """(certified warm starts, assignments solved) since construction,
        over the polygon/line envs of a ragged batch."""
        s = self.t["lsa_stats"].to(torch.int64).sum(0)
        return int(s[0].item()), int(s[1].item())

    # ---------------------------------------------------------------- metrics
    def episode_metrics(self) -> torch.Tensor:
        """[sum of last-episode rewards, sum of last-episode costs, finished
        episodes] over this shard (float64, on device) — the vector the
        distributed runner all-reduces (gsmarl_amd.distributed)."""
        ep = self.t["episode"].to(torch.float64).clamp_min(0).sum()
        s = self.t["ep_last"].to(torch.float64).sum(0)
        return torch.stack([s[0], s[1], ep])
