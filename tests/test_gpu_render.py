"""gsm_render (HIP) against oracle/render_ref.py: frames bit-identical for
navigation, ragged (mixed, padded rows) and rollout-buffer slots, with and
without edges; argument checks. SURVEY.md §8(f) next #4."""
import numpy as np
import pytest
import torch

from oracle import render_ref as rr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _oracle_frames(nf, edge_ptr, edge_index, ids, W, H, sizes, half_width, edges):
    nf = nf.detach().cpu().numpy()
    ep = edge_ptr.detach().cpu().numpy()
    ei = edge_index.detach().cpu().numpy()
    E = nf.shape[1]
    out = []
    for b in ids:
        e = rr.env_edges(ep, ei, b, E) if edges else None
        out.append(rr.render_frame(nf[b], e, W, H, sizes, half_width, edges)[..., :3])
    return np.stack(out)


def _check(got, want):
    got = got.cpu().numpy()
    bad = np.any(got != want, axis=-1)
    assert not bad.any(), (int(bad.sum()), np.argwhere(bad)[:5])


@pytest.mark.parametrize("edges", [True, False])
@pytest.mark.parametrize("kw,W,H", [(dict(n_agents=6, n_envs=8), 160, 120),
                                    (dict(n_agents=24, n_envs=16), 256, 256),
                                    (dict(scenario="mixed", n_agents=12, n_envs=12), 200, 150),
                                    (dict(scenario="polygon", n_agents=5, n_envs=4), 96, 96)])
def test_render_matches_oracle(kw, W, H, edges):
    from gsmarl_amd import EnvConfig, GpuBatchEnv
    env = GpuBatchEnv(EnvConfig(seed=11, **kw), DEV)
    env.reset(seed=11)
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    for _ in range(4):
        env.step(torch.randint(0, 5, (env.B, env.N), dtype=torch.int32, device=DEV, generator=g))
    ids = [0, env.B // 2, env.B - 1]
    frames = env.render(ids, width=W, height=H, edges=edges)
    torch.cuda.synchronize()
    assert frames.shape == (3, H, W, 3) and frames.dtype == torch.uint8
    c = env.cfg
    want = _oracle_frames(env.t["node_feat"], env.t["edge_ptr"], env.t["edge_index"], ids, W, H,
                          (c.agent_size, c.goal_size, c.obstacle_size), c.world_half or 0.0, edges)
    _check(frames, want)
    # something was drawn
    assert (frames != 255).any()
    env.close()


def test_render_rollout_slots_and_bad_ids():
    from gsmarl_amd import EnvConfig, GpuBatchEnv, GraphRolloutBuffer
    from gsmarl_amd.render import render_frames
    env = GpuBatchEnv(EnvConfig(n_agents=3, n_envs=32, seed=2, episode_length=4), DEV)
    buf = GraphRolloutBuffer(env, episode_length=6)
    buf.reset(seed=2)
    acts = torch.randint(0, 5, (6, 32, 3), dtype=torch.int32, device=DEV)
    buf.capture(acts)
    buf.replay()
    frames = buf.render(env=5, width=64, height=64)
    torch.cuda.synchronize()
    assert frames.shape == (7, 64, 64, 3)
    c = env.cfg
    for t in (0, 3, 6):
        want = _oracle_frames(buf.node_feat[t], buf.edge_ptr[t], buf.edge_index[t], [5], 64, 64,
                              (c.agent_size, c.goal_size, c.obstacle_size), c.world_half, True)
        _check(frames[t:t + 1], want)
    # out-of-range env ids: white frames
    white = render_frames(env.t["node_feat"], env.t["edge_ptr"], env.t["edge_index"], [-1, 32], 16, 8)
    assert bool((white == 255).all())
    with pytest.raises(Exception):
        render_frames(env.t["node_feat"], env.t["edge_ptr"], env.t["edge_index"], [0], 0, 8)
    env.close()


def test_env_render_api_and_gif(tmp_path):
    from gsmarl_amd import make_env
    from gsmarl_amd.render import save_gif
    env = make_env("navigation", n_agents=3, n_envs=2, device=DEV)
    env.reset(seed=1)
    imgs = [env.render("rgb_array")[0]]
    for _ in range(3):
        env.step(np.zeros((2, 3), np.int64))
        imgs.append(env.render("rgb_array")[0])
    assert imgs[0].shape == (700, 700, 3) and imgs[0].dtype == np.uint8
    save_gif(np.stack(imgs), tmp_path / "ep.gif", fps=5)
    from PIL import Image
    im = Image.open(tmp_path / "ep.gif")
    assert im.size == (700, 700) and im.n_frames == 4
    env.close()
