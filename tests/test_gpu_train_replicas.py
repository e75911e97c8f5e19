"""Replica training (sac/train_replicas.py) end to end on the MI355X: the real
engine, a probe env, SAC.run_vectorized_training_loop with the replica
aggregator, and the metric vector all-reduced over RCCL -- a one-rank
``nccl`` process group on cuda:0, the hardware leg of the collective the
gloo test (tests/test_train_replicas.py) checks for two ranks on the CPU."""
import copy
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg():
    return {
        "sac": {"gamma": 0.99, "tau": 0.005, "alpha": 0.2, "auto_entropy_tuning": True, "actor_lr": 3e-4,
                "critic_lr": 3e-4, "alpha_lr": 3e-4},
        "q_net": {"hidden_sizes": [32, 32], "hidden_layers_act": "relu", "output_activation": "identity"},
        "policy_net": {"hidden_sizes": [32, 32], "hidden_layers_act": "relu", "output_activation": "identity",
                       "log_std_min": -20, "log_std_max": 2, "action_scale": 1.0},
        "buffer": {"capacity": 4096},
        "train": {"gradient_steps_per_update": 1, "update_frequency": 1, "seed": 5, "batch_size": 16,
                  "warming_steps": 24, "device": "cuda", "precision": "fp32", "graph_chunk": 4},
        "logger": {"enabled": False, "env_name": "probe", "agent_name": "SAC", "log_episode_stats": False,
                   "log_q_values": False, "save_model": {"enabled": False, "path": None}},
    }


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_replica_training_on_the_engine_over_rccl():
    import torch.distributed as dist

    from sac.replicas import METRICS
    from sac.train_replicas import env_factory, train_replica

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        cfg = _cfg()
        out = train_replica(copy.deepcopy(cfg), env_factory("point_mass"), num_envs=4, env_steps=400, every=32,
                            rank=0, device="cuda:0")
    finally:
        dist.destroy_process_group()
    m, agg = out["metrics"], out["aggregate"]
    assert m["gradient_steps"] > 64
    assert agg["world"] == 1 and agg["fields"] == list(METRICS)
    assert agg["aggregations"] == m["gradient_steps"] // 32 + 1
    f = list(METRICS)
    s, mx = agg["last_sum"], agg["last_max"]
    assert s[f.index("steps")] == m["gradient_steps"]  # the engine's own step counter
    assert mx[f.index("wall_s")] > 0
    for k in ("q1_loss", "q2_loss", "policy_loss", "alpha_loss", "alpha"):
        assert s[f.index(k)] is not None and np.isfinite(s[f.index(k)]), k
    assert s == agg["last_mean"]  # one rank: the mean is the sum
