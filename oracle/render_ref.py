"""Frame rasteriser restated in NumPy float32 — the checker for gsm_render.

TEST INFRASTRUCTURE ONLY (the checker); see oracle/batch_ref.py's header.

SURVEY.md §8(f) next #4: the reference renders episodes with the MPE pyglet
viewer (``multiagent/rendering.py``, GSMARL.egg-info/SOURCES.txt:18;
``scripts/render_mpe.py``, SOURCES.txt:30) and ships the resulting GIFs under
``demo/`` (readme.md:64). The viewer source is absent from the reference
tree, so the drawing convention is pinned to those GIFs instead
(tests/golden/make_render_fixture.py extracts a frame; tests/test_render_ref.py
checks this module against it):

* 700 x 700 frames, white background, the camera spans [-L, L]^2 of the world
  (L = the env's half-width: 350 px per unit at 3 agents, 124 at 24), y up;
* discs in entity order (agents, goals/targets, obstacles; later on top), the
  fill and outline colours measured from the GIFs, outline 1.5 px wide;
* the graph's edges as black lines 1 px wide, drawn last.

Per pixel, in float32 (the kernel, gs-marl_amd/csrc/gsm_render.hip, makes the
same operations in the same order without FMA contraction, so frames are
bit-identical):

  sx = (2L)/W, sy = (2L)/H;  x = (px + 0.5)*sx - L;  y = L - (py + 0.5)*sy
  disc e (radius r, type k): d2 = dx*dx + dy*dy with dx = x - ex;
      d2 <= r*r  ->  outline colour if d2 > ri*ri (ri = max(r - 1.5*sx, 0)) else fill
  edge a-b (a < b):  ab = b - a, ap = p - a, t = ap.ab, l2 = ab.ab, w = 0.5*sx
      t <= 0: |ap|^2 <= w*w;  t >= l2: |p - b|^2 <= w*w;
      else: (ap.x*ab.y - ap.y*ab.x)^2 <= (w*w)*l2
"""
from __future__ import annotations

import numpy as np

F = np.float32
# type 0 agent, 1 goal / target, 2 obstacle (node_feat column 6)
FILL = np.array([(159, 159, 223), (64, 64, 64), (128, 128, 128)], dtype=np.uint8)
OUTLINE = np.array([(127, 127, 191), (48, 48, 48), (96, 96, 96)], dtype=np.uint8)
OUTLINE_PX = F(1.5)


def half_width_of(node_rows: np.ndarray, half_width: float) -> np.float32:
    """The frame's half-width: `half_width` if > 0, else sqrt(n_agents / 3)
    in float32 (n_agents = rows of type 0)."""
    if half_width > 0:
        return F(half_width)
    n = int((node_rows[:, 6] == 0).sum())
    return np.sqrt(F(n) / F(3.0)).astype(F)


def render_frame(node_rows: np.ndarray, edges: np.ndarray, width: int, height: int,
                 sizes=(0.05, 0.05, 0.08), half_width: float = 0.0, draw_edges: bool = True) -> np.ndarray:
    """One env's frame. node_rows: [E, 7] float32 node features (pos in
    columns 2-3, type in column 6, -1 = padding); edges: [2, n] local entity
    ids. Returns uint8 [H, W, 4] RGBA."""
    rows = np.asarray(node_rows, dtype=F)
    L = half_width_of(rows, half_width)
    sx = (F(2.0) * L) / F(width)
    sy = (F(2.0) * L) / F(height)
    px = np.arange(width, dtype=F)
    py = np.arange(height, dtype=F)
    x = ((px + F(0.5)) * sx - L)[None, :]
    y = (L - (py + F(0.5)) * sy)[:, None]
    img = np.full((height, width, 3), 255, dtype=np.uint8)
    radii = np.asarray(sizes, dtype=F)
    for e in range(rows.shape[0]):
        k = int(rows[e, 6])
        if k < 0:
            continue
        r = radii[k]
        ri = max(r - OUTLINE_PX * sx, F(0.0))
        dx = x - rows[e, 2]
        dy = y - rows[e, 3]
        d2 = dx * dx + dy * dy
        inside = d2 <= r * r
        ring = inside & (d2 > ri * ri)
        img[inside & ~ring] = FILL[k]
        img[ring] = OUTLINE[k]
    if draw_edges and edges is not None and len(edges) and edges.shape[1]:
        w = F(0.5) * sx
        w2 = w * w
        for a, b in zip(edges[0].tolist(), edges[1].tolist()):
            if a >= b:
                continue
            ax, ay = rows[a, 2], rows[a, 3]
            bx, by = rows[b, 2], rows[b, 3]
            abx, aby = bx - ax, by - ay
            apx, apy = x - ax, y - ay
            t = apx * abx + apy * aby
            l2 = abx * abx + aby * aby
            bpx, bpy = x - bx, y - by
            cross = apx * aby - apy * abx
            on = np.where(t <= F(0.0), apx * apx + apy * apy <= w2,
                          np.where(t >= l2, bpx * bpx + bpy * bpy <= w2, cross * cross <= w2 * l2))
            img[on] = 0
    out = np.empty((height, width, 4), dtype=np.uint8)
    out[..., :3] = img
    out[..., 3] = 255
    return out


def env_edges(edge_ptr: np.ndarray, edge_index: np.ndarray, b: int, n_entities: int) -> np.ndarray:
    """Env b's edges as local entity ids from the batch's packed CSR."""
    lo, hi = int(edge_ptr[b]), int(edge_ptr[b + 1])
    return np.asarray(edge_index[:, lo:hi], dtype=np.int64) - b * n_entities
