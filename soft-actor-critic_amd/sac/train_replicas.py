"""Independent-seed replica training, one process per GPU.

The reference trains ONE learner per ``main.py`` run (reference main.py:43-48
-> sac/agent.py:329-418).  The SAC step does not shard, so N GPUs train N
independent learners: rank r uses seed ``train.seed + r`` for its networks,
device RNG and envs, trains on ``cuda:LOCAL_RANK`` through
``SAC.run_vectorized_training_loop``, and every ``--aggregate-every``
gradient steps the replica metric vector (``sac.replicas.METRICS``: steps,
wall_s, the four losses, alpha, mean return of the last 100 episodes) is
all-reduced over RCCL (``torch.distributed`` backend "nccl" on ROCm) on the
device, with no host synchronisation in the loop.  Rank 0 prints the final
aggregate as one JSON line.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29500 \\
        soft-actor-critic_amd/sac/train_replicas.py --config cfg.yaml \\
        --env point_mass --num-envs 16 --env-steps 200000

Without torchrun it runs one replica in-process.  ``--env`` names one of the
probe envs of ``sac.envs`` or, when gymnasium is importable, any registered
gymnasium id (the reference's own envs).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
from typing import Callable, Optional

import torch

if __package__ in (None, ""):  # run as a script: make `sac` importable
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sac.replicas import ReplicaAggregator, replica_seed  # noqa: E402

PROBE_ENVS = {
    "point_mass": ("OneDPointMassReachEnv", {}),
    "constant_reward": ("ConstantRewardEnv", {}),
    "quadratic_action": ("QuadraticActionRewardEnv", {}),
    "random_obs_binary": ("RandomObsBinaryRewardEnv", {}),
}


def env_factory(name: str) -> Callable[[], object]:
    """A zero-argument env constructor for ``name``: a probe env of sac.envs,
    else a gymnasium id (gymnasium must be importable)."""
    if name in PROBE_ENVS:
        from sac import envs

        cls, kw = PROBE_ENVS[name]
        return lambda: getattr(envs, cls)(**kw)
    try:
        import gymnasium as gym
    except ImportError as e:  # the probe envs need nothing
        raise SystemExit(f"--env {name!r}: not a probe env ({sorted(PROBE_ENVS)}) and gymnasium is not installed") from e
    return lambda: gym.make(name)


def rank_env() -> tuple:
    """(rank, world, local_rank) from the torchrun environment (0, 1, 0 without it)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def train_replica(config: dict, make_env: Callable[[], object], num_envs: int, env_steps: int, every: int,
                  rank: int, device: Optional[str] = None, agent_cls=None, vec_env_cls=None) -> dict:
    """Train this rank's replica and return {"metrics": its loop metrics,
    "aggregate": the all-reduced METRICS summary}.  ``agent_cls`` /
    ``vec_env_cls`` default to sac.agent.SAC / sac.vector_env.SyncVectorEnv
    (tests pass host stubs)."""
    if agent_cls is None:
        from sac.agent import SAC as agent_cls  # noqa: N813
    if vec_env_cls is None:
        from sac.vector_env import SyncVectorEnv as vec_env_cls  # noqa: N813
    cfg = copy.deepcopy(config)
    cfg["train"]["seed"] = replica_seed(cfg["train"]["seed"], rank)
    if device is not None:
        cfg["train"]["device"] = device
    lg = cfg.get("logger", {})
    if lg.get("agent_name"):
        lg["agent_name"] = f"{lg['agent_name']}_rank{rank}"  # per-replica run directories
    vec = vec_env_cls([make_env] * num_envs)
    agent = agent_cls(vec, cfg)
    if getattr(agent, "engine", None) is None:
        # no HIP engine (no MI355X visible, or train.engine_device: cpu): the
        # learner cannot step and there is no CPU fallback -- say so here,
        # before the loop, instead of failing inside it
        from sac import _engine as E

        raise E.EngineUnavailable(f"replica {rank}: replica training needs the HIP engine on an MI355X "
                                  f"(train.device={cfg['train'].get('device')!r}); there is no CPU fallback")
    agg = ReplicaAggregator(agent.engine, every)
    metrics = agent.run_vectorized_training_loop(env_steps, callback=agg, seed=cfg["train"]["seed"])
    return {"metrics": metrics, "aggregate": agg.finish()}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--config", required=True, help="YAML config in the reference's format")
    ap.add_argument("--env", default="point_mass")
    ap.add_argument("--num-envs", type=int, default=16)
    ap.add_argument("--env-steps", type=int, default=100_000)
    ap.add_argument("--aggregate-every", type=int, default=1000, help="gradient steps between all-reduces")
    a = ap.parse_args(argv)
    import yaml

    with open(a.config) as f:
        config = yaml.safe_load(f)
    rank, world, local = rank_env()
    if not torch.cuda.is_available():
        raise SystemExit("train_replicas: no HIP device visible; replica training runs the HIP engine, one "
                         "process per MI355X (there is no CPU fallback)")
    device = f"cuda:{local}"
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL on ROCm: the metric all-reduce only
    try:
        out = train_replica(config, env_factory(a.env), a.num_envs, a.env_steps, a.aggregate_every, rank, device)
    finally:
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"replicas": world, "rank0": out["metrics"], "aggregate": out["aggregate"]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
