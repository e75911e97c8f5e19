"""Vectorised rollout host logic without a GPU: SyncVectorEnv
steps N probe envs exactly like N independent reference-style loops
(agent.py:343-360: step, store (s, a, r, s', terminated or truncated), reset on
done), and the update schedule of the batched driver equals the reference's
per-env-step counting (agent.py:361-364)."""
import numpy as np
import pytest

from sac.agent import due_updates
from sac.envs import OneDPointMassReachEnv, QuadraticActionRewardEnv, RandomObsBinaryRewardEnv
from sac.vector_env import SyncVectorEnv


def _make(kind):
    if kind == "point":
        return lambda: OneDPointMassReachEnv(max_steps=7, action_low=-0.5, action_high=0.5, goal_tolerance=0.2)
    if kind == "randobs":
        return lambda: RandomObsBinaryRewardEnv(obs_dim=3, max_steps=5)
    return lambda: QuadraticActionRewardEnv(max_steps=3)


@pytest.mark.parametrize("kind", ["point", "randobs", "quad"])
@pytest.mark.parametrize("n", [1, 4])
def test_sync_vector_env_matches_independent_loops(kind, n):
    vec = SyncVectorEnv([_make(kind)] * n)
    singles = [_make(kind)() for _ in range(n)]
    obs, _ = vec.reset(seed=11)
    s_obs = np.stack([np.asarray(e.reset(seed=11 + i)[0], np.float32).reshape(-1) for i, e in enumerate(singles)])
    assert np.array_equal(obs, s_obs)
    rng = np.random.default_rng(3)
    n_done = 0
    for _ in range(40):
        act = rng.uniform(-1, 1, (n, vec.act_dim)).astype(np.float32)
        nobs, rew, term, trunc, info = vec.step(act)
        for i, e in enumerate(singles):
            o, r, te, tr, _ = e.step(act[i])
            # the stored transition: true next state and done = terminated or truncated
            assert np.array_equal(info["final_obs"][i], np.asarray(o, np.float32).reshape(-1))
            assert rew[i] == r and term[i] == te and trunc[i] == tr
            if te or tr:
                n_done += 1
                o, _ = e.reset()
            assert np.array_equal(nobs[i], np.asarray(o, np.float32).reshape(-1))
    assert n_done > 0  # autoreset exercised


def test_vector_env_exposes_single_env_spaces():
    vec = SyncVectorEnv([_make("randobs")] * 3)
    assert vec.num_envs == 3 and vec.observation_space.shape == (3,) and vec.action_space.shape == (1,)
    vec.seed_action_spaces(5)
    a = vec.sample_actions()
    assert a.shape == (3, 1) and a.dtype == np.float32
    with pytest.raises(ValueError):
        SyncVectorEnv([])


@pytest.mark.parametrize("update_frequency,grad_steps", [(1, 1), (2, 3), (5, 5), (7, 1)])
@pytest.mark.parametrize("n", [1, 3, 8, 64])
def test_due_updates_equals_per_step_counting(update_frequency, grad_steps, n):
    total = 0
    for _ in range(50):
        ref = sum(grad_steps for t in range(total + 1, total + n + 1) if t % update_frequency == 0)
        assert due_updates(total, total + n, update_frequency, grad_steps) == ref
        total += n
