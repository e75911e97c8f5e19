"""Rollout + training-loop driver throughput on one MI355X.

Three loops over a cheap host env with BipedalWalker-v3's shapes (obs 24, act 4,
1600-step episodes; the dynamics are a random walk, this measures the loop, not
Box2D), C2 networks (2x[256,256], bf16), synthetic data:

  reference   SAC.run_training_loop: per env step one B=1 policy kernel + D2H,
              one replay push, one gradient step (agent.py:343-364)
  vectorized  SAC.run_vectorized_training_loop over N envs: one policy kernel,
              one push and one K-step engine call per vector step
  collect     the vectorised loop with updates disabled (update_frequency > steps)

    python tools/rollout_bench.py [--envs 64] [--steps 20000]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


class Box:
    def __init__(self, n, lo=-np.inf, hi=np.inf):
        self.shape = (n,)
        self.low = np.full(n, lo, np.float32)
        self.high = np.full(n, hi, np.float32)
        self._rng = np.random.default_rng(0)

    def seed(self, s=None):
        self._rng = np.random.default_rng(s)

    def sample(self):
        return self._rng.uniform(-1, 1, self.shape).astype(np.float32)


class WalkerShapedEnv:
    spec = None

    def __init__(self, obs=24, act=4, horizon=1600):
        self.observation_space, self.action_space = Box(obs), Box(act, -1.0, 1.0)
        self.horizon = horizon
        self._rng = np.random.default_rng(0)
        self.t = 0
        self.x = np.zeros(obs, np.float32)

    def reset(self, seed=None, options=None):
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        self.t = 0
        self.x = self._rng.standard_normal(self.x.shape[0]).astype(np.float32)
        return self.x.copy(), {}

    def step(self, a):
        self.t += 1
        self.x = (0.9 * self.x + 0.1 * self._rng.standard_normal(self.x.shape[0])).astype(np.float32)
        r = float(-np.sum(np.square(a)) * 0.01 + 0.1 * self.x[0])
        return self.x.copy(), r, False, self.t >= self.horizon, {}


def cfg(batch=256, warming=256, capacity=1_000_000, update_frequency=1):
    return {
        "sac": {"gamma": 0.99, "tau": 0.005, "alpha": 0.1, "auto_entropy_tuning": True, "actor_lr": 3e-4,
                "critic_lr": 3e-4, "alpha_lr": 3e-4},
        "q_net": {"hidden_sizes": [256, 256], "hidden_layers_act": "relu", "output_activation": "identity"},
        "policy_net": {"hidden_sizes": [256, 256], "hidden_layers_act": "relu", "output_activation": "identity",
                       "log_std_min": -20, "log_std_max": 2, "action_scale": 1.0},
        "buffer": {"capacity": capacity},
        "train": {"gradient_steps_per_update": 1, "update_frequency": update_frequency, "seed": 0, "batch_size": batch,
                  "warming_steps": warming, "device": "cuda", "precision": "bf16", "graph_chunk": 32},
        "logger": {"enabled": False, "env_name": "walker-shaped", "agent_name": "SAC", "log_episode_stats": False,
                   "log_q_values": False, "save_model": {"enabled": False, "path": None}},
    }


def main():
    from sac.agent import SAC
    from sac.vector_env import SyncVectorEnv

    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--ref-seconds", type=float, default=10.0)
    args = ap.parse_args()
    out = {"env": "WalkerShapedEnv (obs 24, act 4, host random walk)", "nets": "2x[256,256] bf16, B=256"}

    # reference-pattern loop: time a bounded number of 1600-step episodes after warm-up
    a = SAC(WalkerShapedEnv(), cfg())
    a.run_training_loop(num_episodes=1, tqdm_disable=True)  # warm-up incl. first gradient steps
    torch.cuda.synchronize()
    s0, g0 = len(a.replay_buffer), a.engine.steps_done
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.ref_seconds:
        a.run_training_loop(num_episodes=1, tqdm_disable=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out["reference_loop"] = {"env_steps_per_s": round((len(a.replay_buffer) - s0) / el, 1),
                             "grad_steps_per_s": round((a.engine.steps_done - g0) / el, 1), "envs": 1}
    del a

    N = args.envs
    for name, every in (("vectorized_loop", 1), ("collect_only", 10 ** 9)):
        v = SAC(SyncVectorEnv([WalkerShapedEnv] * N), cfg(update_frequency=every))
        v.run_vectorized_training_loop(max(N * 8, 512))  # warm-up
        torch.cuda.synchronize()
        g0 = v.engine.steps_done
        t0 = time.perf_counter()
        m = v.run_vectorized_training_loop(args.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[name] = {"env_steps_per_s": round(m["total_env_steps"] / el, 1),
                     "grad_steps_per_s": round((v.engine.steps_done - g0) / el, 1), "envs": N}
        del v
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
