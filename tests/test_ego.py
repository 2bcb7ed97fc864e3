"""Ego-relative node features (gsmarl_amd.ego; InforMARL-style per-agent
view, SURVEY.md a7 [EXT]) against a per-agent loop restatement. Pure tensor
formatting of the kernels' absolute node table, so it runs on CPU tensors."""
import numpy as np
import torch

from gsmarl_amd.ego import EgoView, ego_rows


def _loop(nf, i):
    out = np.zeros_like(nf)
    for b in range(nf.shape[0]):
        vi, pi = nf[b, i, 0:2], nf[b, i, 2:4]
        for e in range(nf.shape[1]):
            v, p, g, t = nf[b, e, 0:2], nf[b, e, 2:4], nf[b, e, 4:6], nf[b, e, 6]
            out[b, e, 0:2] = v - vi
            out[b, e, 2:4] = p - pi
            out[b, e, 4:6] = (g + (p - pi)) if t == 0 else 0.0
            out[b, e, 6] = t
    return out


def test_ego_view_matches_loop():
    rng = np.random.default_rng(0)
    B, N, No = 3, 4, 2
    E = 2 * N + No
    nf = rng.normal(size=(B, E, 7)).astype(np.float32)
    nf[:, N:, 0:2] = 0
    nf[:, N:, 4:6] = 0
    nf[:, :, 6] = np.array([0] * N + [1] * N + [2] * No, np.float32)
    t = torch.from_numpy(nf)
    view = EgoView(t, N)
    allv = view.all().numpy()
    assert allv.shape == (B, N, E, 7)
    for i in range(N):
        want = _loop(nf, i)
        assert np.allclose(view[i].numpy(), want, atol=1e-6)
        assert np.allclose(allv[:, i], want, atol=1e-6)
        assert np.allclose(ego_rows(t, torch.full((B,), i)).numpy(), want, atol=1e-6)
    # the ego agent sees itself at the origin with zero relative velocity
    for i in range(N):
        assert np.all(allv[:, i, i, 0:4] == 0)
