"""The renderer's checker (oracle/render_ref.py)
pinned to the reference's own demo GIFs (tests/golden/demo_nav{3,24}_f0.png:
frame 0 of demo/navigation/{3,24}agents.gif, readme.md:64, extracted by
tests/golden/make_render_fixture.py). The reference's viewer source is absent,
so what is pinned is the drawing convention: palette, camera [-L, L]^2 with
L = sqrt(N/3) (scale W / 2L), disc radii = entity sizes with a 1.5 px ring.
Anti-aliasing of the pyglet frames is not reproduced (the checks allow 1 px)."""
import numpy as np
import pytest
from pathlib import Path
from scipy import ndimage

from oracle import render_ref as rr

GOLD = Path(__file__).resolve().parent / "golden"


def _frame(n):
    from PIL import Image
    return np.asarray(Image.open(GOLD / f"demo_nav{n}_f0.png").convert("RGB")).astype(np.int64)


def _isolated_radii(img, color, min_area):
    m = np.all(img == color, axis=-1)
    lab, n = ndimage.label(m)
    areas = ndimage.sum(m, lab, range(1, n + 1))
    return np.sqrt(np.array([a for a in areas if a >= min_area]) / np.pi)


@pytest.mark.parametrize("n_agents", [3, 24])
def test_palette_and_scale_match_demo_gifs(n_agents):
    img = _frame(n_agents)
    H, W, _ = img.shape
    assert (H, W) == (700, 700)
    assert (np.all(img == 255, axis=-1)).mean() > 0.9              # white background
    L = np.sqrt(n_agents / 3.0)
    scale = W / (2 * L)                                            # px per world unit
    sizes = (0.05, 0.05)                                           # agent, goal
    for k in (0, 1):                                               # fill colours, measured
        fill = rr.FILL[k]
        assert np.all(img == fill, axis=-1).sum() > 200, k
        want = sizes[k] * scale - float(rr.OUTLINE_PX)             # fill radius in px
        r = _isolated_radii(img, fill, min_area=0.8 * np.pi * want ** 2)
        assert len(r) >= 1, k
        assert np.all(np.abs(r - want) <= 1.0), (k, r, want)
    # ring colours present around the discs
    for k in (0, 1, 2):
        assert np.all(img == rr.OUTLINE[k], axis=-1).sum() > 20, k
    # edge lines: anti-aliased dark greys off the palette
    grey = (img[..., 0] == img[..., 1]) & (img[..., 1] == img[..., 2]) & (img[..., 0] < 200)
    pal = np.zeros(grey.shape, bool)
    for c in list(rr.FILL) + list(rr.OUTLINE):
        pal |= np.all(img == c, axis=-1)
    assert (grey & ~pal).sum() > 100


def test_oracle_geometry_small():
    rows = np.zeros((3, 7), np.float32)
    rows[0, [2, 3, 6]] = (0.0, 0.0, 0)        # agent at the centre
    rows[1, [2, 3, 6]] = (0.5, 0.5, 1)        # goal
    rows[2, [2, 3, 6]] = (0.0, 0.0, -1)       # padding: not drawn
    img = rr.render_frame(rows, np.array([[0, 1], [1, 0]]), 100, 100, half_width=1.0)
    assert img.shape == (100, 100, 4) and np.all(img[..., 3] == 255)
    assert tuple(img[50, 50, :3]) == tuple(rr.FILL[0])             # pixel centre (0.01, -0.01)
    assert tuple(img[0, 0, :3]) == (255, 255, 255)
    # the goal disc centre (0.5, 0.5) -> pixel column 75, row 25
    assert tuple(img[24, 74, :3]) in (tuple(rr.FILL[1]), (0, 0, 0))
    # a point on the segment (0,0)-(0.5,0.5) away from both discs is black
    assert tuple(img[35, 64, :3]) == (0, 0, 0)
    # ring pixels exist at the agent's edge (radius 0.05 = 2.5 px)
    ring = np.all(img[..., :3] == rr.OUTLINE[0], axis=-1)
    assert ring.sum() > 0
    # no edges: no black pixels
    img2 = rr.render_frame(rows, None, 100, 100, half_width=1.0, draw_edges=False)
    assert not np.any(np.all(img2[..., :3] == 0, axis=-1))


def test_default_half_width_counts_agents():
    rows = np.zeros((5, 7), np.float32)
    rows[:3, 6] = 0
    rows[3:, 6] = 2
    assert rr.half_width_of(rows, 0.0) == np.float32(1.0)
    rows[:, 6] = 0
    assert rr.half_width_of(rows, 0.0) == np.sqrt(np.float32(5) / np.float32(3))
    assert rr.half_width_of(rows, 2.5) == np.float32(2.5)
