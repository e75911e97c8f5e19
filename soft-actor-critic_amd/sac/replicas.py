"""Independent-seed replicas, one process per GPU (the SAC step
does not shard — each step depends on the previous step's parameters, so
multi-GPU = N independent learners).  The only collective is the periodic
metric aggregation over RCCL (``torch.distributed`` backend "nccl" on ROCm),
a few float64 scalars per reduction.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

# order of the aggregated metric vector
METRICS = ("steps", "wall_s", "q1_loss", "q2_loss", "policy_loss", "alpha_loss", "alpha", "mean_return")


def replica_seed(base_seed: int, rank: int) -> int:
    """Seed of replica ``rank``: base + rank (network init, device RNG, env)."""
    return int(base_seed) + int(rank)


def aggregate_metrics(values: Sequence[float], group=None, device: Optional[torch.device] = None):
    """All-reduce one replica's metric vector -> (sum, mean, max) over replicas.

    ``steps`` and ``wall_s`` are summed / maxed; the losses are averaged.  Works
    on gloo (CPU tensors) and nccl/RCCL (device tensors)."""
    import torch.distributed as dist

    v = torch.tensor(list(values), dtype=torch.float64, device=device)
    world = dist.get_world_size(group)
    s = v.clone()
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    m = v.clone()
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return {"sum": s.tolist(), "mean": (s / world).tolist(), "max": m.tolist(), "world": world}


def timed_region(run, sync, device: Optional[torch.device] = None, group=None) -> float:
    """Wall time of ``run()`` bracketed by (barrier + ``sync()``) on both sides,
    MAX over ranks (the bench contract; single process when not initialised)."""
    import time

    import torch.distributed as dist

    on = dist.is_available() and dist.is_initialized()
    sync()
    if on:
        dist.barrier(group)
    sync()
    t0 = time.perf_counter()
    run()
    sync()
    if on:
        dist.barrier(group)
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if on:
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=group)
    return float(el.item())


def aggregate_throughput(steps: int, wall_s: float, group=None, device=None) -> float:
    """Whole-job steps/s: total steps of all replicas / slowest replica's time."""
    agg = aggregate_metrics([steps, wall_s], group, device)
    return agg["sum"][0] / agg["max"][1]
