"""A deterministic probe environment shared by tests/golden/make_golden.py (run
against the reference's ``run_training_loop``) and the GPU loop tests (run
against this repo's loops).  Observations, rewards and episode ends depend only
on the step and episode counters -- never on the action -- so both sides push
the same (s, r, s', done) rows whatever their policies sample.

Gymnasium-style API: ``reset(seed=None) -> (obs, info)``, ``step(a) -> (obs,
reward, terminated, truncated, info)``, ``observation_space`` / ``action_space``
with ``shape``, ``seed`` and ``sample``."""
from __future__ import annotations

import numpy as np


class _Space:
    def __init__(self, n):
        self.shape = (n,)

    def seed(self, s=None):
        return [s]

    def sample(self):
        return np.zeros(self.shape, np.float32)


class DetEnv:
    spec = None

    def __init__(self, obs_dim: int, act_dim: int, ep_lengths=(7, 4, 11, 5), truncate_at: int = 9, offset: int = 0):
        self.observation_space = _Space(obs_dim)
        self.action_space = _Space(act_dim)
        self.ep_lengths = tuple(ep_lengths)
        self.truncate_at = truncate_at
        self.episode = offset - 1
        self.t = 0

    def _obs(self) -> np.ndarray:
        k = np.arange(self.observation_space.shape[0], dtype=np.float64)
        return np.sin(0.37 * (k + 1) * (self.t + 1) + 0.11 * self.episode).astype(np.float32)

    def reset(self, seed=None, options=None):
        self.episode += 1
        self.t = 0
        return self._obs(), {}

    def step(self, action):
        self.t += 1
        length = self.ep_lengths[self.episode % len(self.ep_lengths)]
        terminated = self.t >= length
        truncated = (not terminated) and self.t >= self.truncate_at
        reward = float(np.cos(0.5 * self.t) + 0.01 * self.episode)
        return self._obs(), reward, bool(terminated), bool(truncated), {}

    def close(self):
        pass
