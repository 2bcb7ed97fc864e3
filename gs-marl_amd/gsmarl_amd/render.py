"""Episode frames and GIF export.

Stands in for the reference's pyglet viewer (``multiagent/rendering.py``,
GSMARL.egg-info/SOURCES.txt:18) as driven by ``scripts/render_mpe.py``
(SOURCES.txt:30) to make the ``demo/`` GIFs (readme.md:64). Frames are drawn
on the GPU by ``gsm_render`` from what the env already wrote — node-feature
rows and the packed edge list — so the current state of any env, or any slot
of a ``GraphRolloutBuffer``, can be rendered without a host round trip; the
drawing convention is pinned to the demo GIFs (oracle/render_ref.py).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import torch

from . import _lib


def render_frames(node_feat: torch.Tensor, edge_ptr: Optional[torch.Tensor], edge_index: Optional[torch.Tensor],
                  env_ids, width: int = 700, height: int = 700, sizes: Sequence[float] = (0.05, 0.05, 0.08),
                  half_width: float = 0.0, edges: bool = True) -> torch.Tensor:
    """RGB frames uint8 [n, height, width, 3] of envs ``env_ids`` of a batch
    (node_feat [B, E, 7] f32; edge_ptr [B+1] int64; edge_index [2, cap] int32,
    all on one ROCm device). half_width <= 0: each env's sqrt(n_agents / 3)."""
    dev = node_feat.device
    if dev.type != "cuda":
        raise _lib.GsmError("render_frames needs a ROCm GPU (oracle/render_ref.py is the CPU checker)")
    if node_feat.dtype != torch.float32 or node_feat.dim() != 3 or node_feat.shape[-1] != 7:
        raise ValueError("node_feat: float32 [B, E, 7]")
    nf = node_feat.contiguous()
    ids = torch.as_tensor(env_ids, dtype=torch.int32, device=dev).reshape(-1).contiguous()
    n = ids.numel()
    out = torch.empty(n, height, width, 4, dtype=torch.uint8, device=dev)
    flags = 0
    cap = 0
    if edges:
        if edge_ptr is None or edge_index is None:
            raise ValueError("edges=True needs edge_ptr and edge_index")
        if edge_ptr.dtype != torch.int64 or edge_index.dtype != torch.int32 or not edge_index.is_contiguous():
            raise ValueError("edge_ptr int64, edge_index contiguous int32 [2, cap]")
        flags |= _lib.RENDER_EDGES
        cap = edge_index.shape[1]

    def ptr(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    lib = _lib.load()
    rc = lib.gsm_render(ptr(nf), int(nf.shape[0]), int(nf.shape[1]), ptr(edge_ptr) if edges else None,
                        ptr(edge_index) if edges else None, int(cap), ptr(ids), int(n), float(half_width),
                        float(sizes[0]), float(sizes[1]), float(sizes[2]), int(width), int(height), flags,
                        ptr(out), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    _lib.check(lib, rc, None, "gsm_render")
    return out[..., :3]


def save_gif(frames, path, fps: float = 10.0) -> None:
    """Write frames ([T, H, W, 3] uint8, tensor or array) as a looping GIF
    (Pillow's encoder)."""
    from PIL import Image
    import numpy as np
    arr = frames.detach().cpu().numpy() if isinstance(frames, torch.Tensor) else np.asarray(frames)
    imgs = [Image.fromarray(np.ascontiguousarray(f)) for f in arr]
    imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=int(round(1000.0 / fps)), loop=0)
