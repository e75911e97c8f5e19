"""Probe environments (behaviour of reference ``sac/envs.py``), used as
closed-form end-to-end checks of the engine.

gymnasium is optional: when it is absent a minimal ``Box`` / ``Env`` pair with
the same attributes (shape/low/high/seed/sample, ``np_random``) stands in.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    import gymnasium as _gym
    from gymnasium import spaces as _spaces

    _Env = _gym.Env
    Box = _spaces.Box
except Exception:  # gymnasium absent (this image)
    class Box:
        def __init__(self, low, high, shape, dtype=np.float32):
            self.shape = tuple(shape)
            self.dtype = dtype
            self.low = np.full(self.shape, low, dtype=dtype)
            self.high = np.full(self.shape, high, dtype=dtype)
            self._rng = np.random.default_rng()

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

    class _Env:
        spec = None
        np_random = np.random.default_rng()

        def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
            if seed is not None:
                self.np_random = np.random.default_rng(seed)

        def close(self):
            pass


def _unbounded(n):
    return Box(low=-np.inf, high=np.inf, shape=(n,), dtype=np.float32)


class ConstantRewardEnv(_Env):
    """Reward is constant; episodes last ``max_steps`` (envs.py:15-46).
    With max_steps=1 every transition is terminal, so y == r exactly."""

    def __init__(self, reward: float = 1.0, max_steps: int = 1):
        super().__init__()
        self.constant_reward = float(reward)
        self.max_steps = int(max_steps)
        self.action_space = Box(low=-1.0, high=1.0, shape=(1,), dtype=np.float32)
        self.observation_space = _unbounded(1)
        self.current_step = 0
        self.episode_reward = 0.0

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        super().reset(seed=seed)
        self.current_step, self.episode_reward = 0, 0.0
        return np.zeros(1, dtype=np.float32), {}

    def step(self, action):
        self.current_step += 1
        self.episode_reward += self.constant_reward
        terminated = self.current_step >= self.max_steps
        info = {"episode": {"r": self.episode_reward, "l": self.current_step}} if terminated else {}
        return np.zeros(1, dtype=np.float32), self.constant_reward, terminated, False, info


class QuadraticActionRewardEnv(_Env):
    """One-step bandit, r = -(clip(a) - target)^2 (envs.py:57-98)."""

    def __init__(self, target: float = 0.5, action_low: float = -1.0, action_high: float = 1.0, max_steps: int = 1):
        super().__init__()
        self.target = float(target)
        self.max_steps = int(max_steps)
        self.action_space = Box(low=action_low, high=action_high, shape=(1,), dtype=np.float32)
        self.observation_space = _unbounded(1)
        self.current_step = 0
        self.episode_reward = 0.0

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        super().reset(seed=seed)
        self.current_step, self.episode_reward = 0, 0.0
        return np.zeros(1, dtype=np.float32), {}

    def step(self, action):
        self.current_step += 1
        a = np.clip(action[0], self.action_space.low[0], self.action_space.high[0])
        reward = -((a - self.target) ** 2)
        self.episode_reward += reward
        terminated = self.current_step >= self.max_steps
        info = {"action": a}
        if terminated:
            info["episode"] = {"r": self.episode_reward, "l": self.current_step}
        return np.zeros(1, dtype=np.float32), reward, terminated, False, info


class RandomObsBinaryRewardEnv(_Env):
    """Uniform-noise observations; r = +1 iff |a| <= threshold (envs.py:109-150)."""

    def __init__(self, obs_dim: int = 4, threshold: float = 0.2, max_steps: int = 1):
        super().__init__()
        self.obs_dim = int(obs_dim)
        self.threshold = float(threshold)
        self.max_steps = int(max_steps)
        self.action_space = Box(low=-1.0, high=1.0, shape=(1,), dtype=np.float32)
        self.observation_space = _unbounded(self.obs_dim)
        self.current_step = 0
        self.episode_reward = 0.0

    def _obs(self):
        return self.np_random.uniform(low=-1.0, high=1.0, size=self.obs_dim).astype(np.float32)

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        super().reset(seed=seed)
        self.current_step, self.episode_reward = 0, 0.0
        return self._obs(), {}

    def step(self, action):
        self.current_step += 1
        a = float(action[0])
        reward = 1.0 if abs(a) <= self.threshold else -1.0
        terminated = self.current_step >= self.max_steps
        info = {"action": a}
        if terminated:
            info["episode"] = {"r": self.episode_reward, "l": self.current_step}
        return self._obs(), reward, terminated, False, info


class OneDPointMassReachEnv(_Env):
    """1-D point mass driven toward a goal (envs.py:161-222)."""

    def __init__(self, start_pos: float = 0.0, goal_pos: float = 1.0, max_steps: int = 50, dt: float = 1.0,
                 action_low: float = -0.1, action_high: float = 0.1, step_penalty: float = -0.01,
                 goal_reward: float = 1.0, goal_tolerance: float = 0.05):
        super().__init__()
        self.start_pos, self.goal_pos = float(start_pos), float(goal_pos)
        self.max_steps, self.dt = int(max_steps), float(dt)
        self.step_penalty, self.goal_reward = float(step_penalty), float(goal_reward)
        self.goal_tolerance = float(goal_tolerance)
        self.action_space = Box(low=action_low, high=action_high, shape=(1,), dtype=np.float32)
        self.observation_space = _unbounded(1)
        self.current_step = 0
        self.pos = 0.0
        self.episode_reward = 0.0

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        super().reset(seed=seed)
        self.current_step, self.pos, self.episode_reward = 0, self.start_pos, 0.0
        return np.array([self.pos], dtype=np.float32), {}

    def step(self, action):
        self.current_step += 1
        a = float(np.clip(action[0], self.action_space.low[0], self.action_space.high[0]))
        self.pos += a * self.dt
        reward = self.step_penalty
        reached = abs(self.pos - self.goal_pos) <= self.goal_tolerance
        if reached:
            reward += self.goal_reward
        self.episode_reward += reward
        truncated = self.current_step >= self.max_steps
        info = {"action": a}
        if reached or truncated:
            info["episode"] = {"r": self.episode_reward, "l": self.current_step}
        return np.array([self.pos], dtype=np.float32), reward, reached, truncated, info


__all__ = ["ConstantRewardEnv", "QuadraticActionRewardEnv", "RandomObsBinaryRewardEnv", "OneDPointMassReachEnv"]
