"""CPU stand-in for GpuBatchEnv used ONLY by tests/test_bench_launcher.py to
drive bench.py's launcher and rank body without a GPU (`--selftest-env`).

It keeps the bookkeeping the bench relies on — per-env step counters with
auto-reset at the episode length, episode counters, last-episode totals, the
CSR edge_ptr and graph slots replayed by step count — and no physics. The
last-episode reward of global env g is -(g + 1), so the all-reduced metric sum
tells which global envs each rank owned.
"""
from types import SimpleNamespace

import torch


class StubEnv:
    def __init__(self, cfg, device):
        self.cfg = cfg
        self.B, self.N = cfg.n_envs, cfg.n_agents
        self.sizes = SimpleNamespace(envs_per_block=16)
        gid = torch.arange(cfg.env_base, cfg.env_base + self.B, dtype=torch.float32)
        self._ep_reward = -(gid + 1)
        self.t = dict(
            step_count=torch.zeros(self.B, dtype=torch.int32),
            episode=torch.full((self.B,), -1, dtype=torch.int32),
            ep_last=torch.zeros(self.B, 2, dtype=torch.float32),
            edge_ptr=torch.arange(self.B + 1, dtype=torch.int64) * 2,
            env_shape=torch.full((self.B,), self.N, dtype=torch.int32),
        )
        self.slots = {}
        self.steps_run = 0

    def reset(self, seed=None, sync_edges=True):
        self.t["step_count"].zero_()
        self.t["episode"].fill_(0)

    def step(self, actions, sync_edges=True):
        self.steps_run += 1
        sc = self.t["step_count"]
        sc += 1
        done = sc >= self.cfg.episode_length
        if bool(done.any()):
            self.t["ep_last"][done, 0] = self._ep_reward[done]
            self.t["episode"][done] += 1
            sc[done] = 0

    def capture(self, actions, n_steps, timing=False, slot=0, kernels="both", time_ends=False):
        self.slots[slot] = (actions, int(n_steps))

    def replay(self, slot=0):
        actions, n = self.slots[slot]
        for j in range(n):
            self.step(actions[j % actions.shape[0]])

    def episode_metrics(self):
        ep = self.t["episode"].to(torch.float64).clamp_min(0).sum()
        s = self.t["ep_last"].to(torch.float64).sum(0)
        return torch.stack([s[0], s[1], ep])

    def close(self):
        pass


def make_env(cfg, device):
    return StubEnv(cfg, device)
