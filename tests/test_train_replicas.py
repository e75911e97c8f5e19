"""Replica training beyond the bench (sac/train_replicas.py) on the
CPU: two gloo ranks each train an independent-seed learner through the
vectorised loop's per-step callback, with the engine stubbed (host tensors,
as tests/test_bench_ranks.py does for bench.py).  Checked: rank seeds are
base + rank, the replica metric vector METRICS is all-reduced every
``every`` gradient steps and once at the end, and the aggregate holds the
summed steps, the slowest rank's wall time and the averaged losses, alpha and
mean return."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sac.replicas import METRICS


class _StubEngine:
    def __init__(self, rank):
        self.rng_step = torch.zeros(1, dtype=torch.int64)
        self.stats = torch.tensor([1.0 + rank, 2.0, -0.5, 0.1, 0.0, 0.0], dtype=torch.float32)
        self.alpha_state = torch.tensor([-2.3, 0.1 * (rank + 1), 0.0, 0.0], dtype=torch.float64)


class _StubVecEnv:
    def __init__(self, fns):
        self.num_envs = len(fns)


class _StubAgent:
    """SAC's construction and loop contract without the engine: 4 gradient
    steps per vector step; the average return is 10 (rank + 1)."""

    def __init__(self, vec_env, config):
        self.config = config
        self.rank = config["train"]["seed"] - 42
        self.engine = _StubEngine(self.rank)
        self.N = vec_env.num_envs

    def run_vectorized_training_loop(self, total_env_steps, callback=None, seed=None):
        assert seed == self.config["train"]["seed"]
        env = grad = 0
        while env < total_env_steps:
            env += self.N
            grad += 4
            self.engine.rng_step += 4
            callback({"env_steps": env, "gradient_steps": grad, "episodes": env // 10,
                      "avg_return": 10.0 * (self.rank + 1)})
        return {"total_env_steps": env, "gradient_steps": grad}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sac.train_replicas import train_replica

        cfg = {"train": {"seed": 42, "device": "cpu"}, "logger": {"agent_name": "SAC"}}
        r = train_replica(cfg, lambda: None, num_envs=8, env_steps=400, every=16, rank=rank,
                          agent_cls=_StubAgent, vec_env_cls=_StubVecEnv)
        out[rank] = r
    finally:
        dist.destroy_process_group()


def test_replica_training_aggregates_over_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert set(out.keys()) == {0, 1}
    f = list(METRICS)
    for r in range(world):
        m, agg = out[r]["metrics"], out[r]["aggregate"]
        assert m["total_env_steps"] == 400 and m["gradient_steps"] == 200  # 50 vector steps x 4
        assert agg["world"] == world and agg["fields"] == f
        # every 16 gradient steps (12 crossings in 200) + the final aggregation
        assert agg["aggregations"] == 200 // 16 + 1
        s, mean, mx = agg["last_sum"], agg["last_mean"], agg["last_max"]
        assert s[f.index("steps")] == 2 * 200
        assert mx[f.index("wall_s")] > 0
        assert mean[f.index("q1_loss")] == pytest.approx(1.5)      # ranks 1.0 and 2.0
        assert mean[f.index("alpha")] == pytest.approx(0.15)       # ranks 0.1 and 0.2
        assert mean[f.index("mean_return")] == pytest.approx(15.0)  # ranks 10 and 20
        assert mx[f.index("mean_return")] == pytest.approx(20.0)


def test_replica_seed_and_logger_name_per_rank():
    from sac.train_replicas import train_replica

    cfg = {"train": {"seed": 42, "device": "cpu"}, "logger": {"agent_name": "SAC"}}
    seen = {}

    class Rec(_StubAgent):
        def __init__(self, vec_env, config):
            super().__init__(vec_env, config)
            seen["seed"], seen["name"] = config["train"]["seed"], config["logger"]["agent_name"]

    train_replica(cfg, lambda: None, 2, 10, 1000, rank=3, agent_cls=Rec, vec_env_cls=_StubVecEnv)
    assert seen == {"seed": 45, "name": "SAC_rank3"}
    assert cfg["train"]["seed"] == 42  # the caller's config is not modified


class _NoEngineAgent(_StubAgent):
    """A rank whose learner never built the engine (an agent on a host without
    a HIP device): the loop ran no gradient step and the engine is None."""

    def __init__(self, vec_env, config):
        super().__init__(vec_env, config)
        self.engine = None


def test_real_agent_on_cpu_is_refused_clearly():
    """The real sac.agent.SAC on a host without a GPU (engine None): train_replica
    raises EngineUnavailable up front, not an AttributeError from the
    aggregator."""
    import copy

    from _fixtures import load
    from sac import _engine as E

    _, meta = load("c1_auto")
    cfg = copy.deepcopy(meta["cfg"])
    cfg["train"]["device"] = "cpu"
    cfg["train"]["engine_device"] = "cpu"
    cfg["logger"]["enabled"] = False
    from sac.train_replicas import train_replica

    with pytest.raises(E.EngineUnavailable, match="no CPU fallback"):
        train_replica(cfg, __import__("sac.train_replicas", fromlist=["env_factory"]).env_factory("point_mass"),
                      num_envs=2, env_steps=8, every=4, rank=0)


def test_aggregator_without_engine_and_without_returns():
    """ReplicaAggregator with no engine builds the metric vector from the loop's
    host counters (NaN losses), and a rank without a finished episode leaves
    mean_return out of the reduction instead of turning it NaN."""
    from sac.replicas import ReplicaAggregator

    agg = ReplicaAggregator(None, every=4)
    agg({"env_steps": 8, "gradient_steps": 8, "episodes": 0, "avg_return": float("nan")})
    out = agg.finish()
    f = list(METRICS)
    assert out["aggregations"] == 2
    assert out["last_sum"][f.index("steps")] == 8
    assert out["last_sum"][f.index("q1_loss")] is None
    assert out["last_sum"][f.index("mean_return")] is None and out["last_max"][f.index("mean_return")] is None
    assert out["last_sum"][f.index("return_ranks")] == 0


def _worker_uneven(rank, world, port, out):
    """Rank 1 has not finished an episode (avg_return NaN): the aggregate's
    mean_return is rank 0's alone, not NaN."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sac.replicas import ReplicaAggregator

        agg = ReplicaAggregator(_StubEngine(rank), every=4)
        agg({"env_steps": 8, "gradient_steps": 8, "episodes": 1 - rank,
             "avg_return": 7.0 if rank == 0 else float("nan")})
        out[rank] = agg.finish()
    finally:
        dist.destroy_process_group()


def test_mean_return_over_ranks_with_episodes():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_uneven, args=(world, port, out), nprocs=world, join=True)
    f = list(METRICS)
    for r in range(world):
        a = out[r]
        assert a["last_mean"][f.index("mean_return")] == pytest.approx(7.0)
        assert a["last_max"][f.index("mean_return")] == pytest.approx(7.0)
        assert a["last_sum"][f.index("return_ranks")] == 1
        assert a["last_mean"][f.index("q1_loss")] == pytest.approx(1.5)
