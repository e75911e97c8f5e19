"""Vectorised environments for batched rollouts.

The reference steps ONE environment per loop iteration (agent.py:343-377): one
B=1 policy forward, one device->host copy and one replay ``push`` per env step.
``SyncVectorEnv`` steps N copies in lockstep so the agent can select N actions
with one policy kernel and append N transitions with one H2D copy + one push
kernel (``SAC.run_vectorized_training_loop``).

Semantics follow ``gymnasium.vector.SyncVectorEnv`` with SAME-STEP autoreset:
an env whose episode ended is reset inside ``step``; the observation it ended
on is returned in ``infos["final_obs"]`` (which holds the true next state of
EVERY env, equal to the returned observation where no episode ended), so the
stored transition is ``(obs, action, reward, final_obs[i], terminated|truncated)``
exactly as the reference's per-env loop stores it (agent.py:352-356).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np


class SyncVectorEnv:
    def __init__(self, env_fns: Sequence[Callable[[], object]]):
        if len(env_fns) == 0:
            raise ValueError("SyncVectorEnv needs at least one environment")
        self.envs: List[object] = [fn() for fn in env_fns]
        self.num_envs = len(self.envs)
        self.single_observation_space = self.envs[0].observation_space
        self.single_action_space = self.envs[0].action_space
        # attributes SAC reads from a single env (observation/action sizes, spec)
        self.observation_space = self.single_observation_space
        self.action_space = self.single_action_space
        self.spec = getattr(self.envs[0], "spec", None)
        self.obs_dim = int(np.prod(self.single_observation_space.shape))
        self.act_dim = int(np.prod(self.single_action_space.shape))
        self._obs = np.zeros((self.num_envs, self.obs_dim), np.float32)

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        """Reset every env; env i is seeded with ``seed + i`` (gymnasium's rule)."""
        infos = []
        for i, env in enumerate(self.envs):
            o, info = env.reset(seed=None if seed is None else seed + i)
            self._obs[i] = np.asarray(o, np.float32).reshape(-1)
            infos.append(info)
        return self._obs.copy(), {"env_infos": infos}

    def seed_action_spaces(self, seed: int) -> None:
        for i, env in enumerate(self.envs):
            env.action_space.seed(seed + i)

    def sample_actions(self) -> np.ndarray:
        return np.stack([np.asarray(env.action_space.sample(), np.float32).reshape(-1) for env in self.envs])

    def step(self, actions):
        actions = np.asarray(actions, np.float32).reshape(self.num_envs, self.act_dim)
        n = self.num_envs
        rewards = np.zeros(n, np.float64)
        terminated = np.zeros(n, bool)
        truncated = np.zeros(n, bool)
        final_obs = np.empty((n, self.obs_dim), np.float32)
        infos = []
        for i, env in enumerate(self.envs):
            o, r, te, tr, info = env.step(actions[i])
            final_obs[i] = np.asarray(o, np.float32).reshape(-1)
            rewards[i], terminated[i], truncated[i] = float(r), bool(te), bool(tr)
            if te or tr:
                o, _ = env.reset()
            self._obs[i] = np.asarray(o, np.float32).reshape(-1)
            infos.append(info)
        return self._obs.copy(), rewards, terminated, truncated, {"final_obs": final_obs, "env_infos": infos}

    def close(self) -> None:
        for env in self.envs:
            close = getattr(env, "close", None)
            if close is not None:
                close()


__all__ = ["SyncVectorEnv"]
