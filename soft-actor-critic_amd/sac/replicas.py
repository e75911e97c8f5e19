"""Independent-seed replicas, one process per GPU (the SAC step
does not shard — each step depends on the previous step's parameters, so
multi-GPU = N independent learners).  The only collective is the periodic
metric aggregation over RCCL (``torch.distributed`` backend "nccl" on ROCm),
a few float64 scalars per reduction.

``replica_train`` is the replica training entry point: it trains this rank's
learner in blocks of ``every`` gradient steps (graph-replayed) and after each
block all-reduces the replica metric vector ("every R steps (e.g.
1,000)").  The vector is built and reduced on the device, on the training
stream's order, with no host synchronisation: training never waits for the
host, only (on the device) for the tens-of-bytes all-reduce.
"""
from __future__ import annotations

import math
import time
from typing import List, Optional, Sequence, Tuple

import torch

# order of the replica metric vector, host (aggregate_metrics) and
# device (metric_vector / replica_train / ReplicaAggregator) forms alike
# mean_return is reduced over the ranks that have finished an episode only:
# the vector carries the return (0 on a rank without one) and the 0/1 flag
# "return_ranks", so one slow rank's NaN does not hide the other ranks'
# returns; the host view divides by the flag count (None while it is 0)
METRICS = ("steps", "wall_s", "q1_loss", "q2_loss", "policy_loss", "alpha_loss", "alpha", "mean_return",
           "return_ranks")
I_RET, I_NRET = METRICS.index("mean_return"), METRICS.index("return_ranks")
REPLICA_METRICS = METRICS


def replica_seed(base_seed: int, rank: int) -> int:
    """Seed of replica ``rank``: base + rank (network init, device RNG, env)."""
    return int(base_seed) + int(rank)


def _initialised() -> bool:
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def _collective_device() -> Optional[torch.device]:
    """Where a host-built metric vector must live for the default process
    group's collectives: this process's HIP device under RCCL ("nccl", which
    rejects CPU tensors), the host otherwise (gloo, or no process group)."""
    import torch.distributed as dist

    if _initialised() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return None


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


def metric_vector(engine, wall_s: float = 0.0, mean_return: float = float("nan"),
                  steps: Optional[int] = None) -> torch.Tensor:
    """METRICS of the engine's last step as a float64 device tensor: the step
    counter, losses and alpha come from the engine's own buffers by device ops
    (no host read); the host scalars wall_s and mean_return enter as fill
    kernels (torch.full: a kernel argument, not a copy), so nothing waits.
    engine None (a learner that never built the HIP engine, e.g. no gradient
    step was due yet): a host vector with the loop's step count ``steps`` and
    NaN losses and alpha."""
    has_ret = math.isfinite(mean_return)
    ret = [float(mean_return) if has_ret else 0.0, 1.0 if has_ret else 0.0]
    if engine is None:
        nan = float("nan")
        return torch.tensor([float(steps or 0), float(wall_s), nan, nan, nan, nan, nan] + ret, dtype=torch.float64,
                            device=_collective_device())
    dev = engine.stats.device
    host = lambda x: torch.full((1,), float(x), dtype=torch.float64, device=dev)  # noqa: E731
    return torch.cat([engine.rng_step.double().reshape(1), host(wall_s), engine.stats[:4].double(),
                      engine.alpha_state[1:2].double(), host(ret[0]), host(ret[1])])


def aggregate_device(v: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sum, max) over replicas of a device vector, without a host sync: with
    RCCL the collectives run on the process group's stream after the current
    stream's work, and the current stream waits for them on the device."""
    import torch.distributed as dist

    s, m = v.clone(), v.clone()
    # the max of mean_return runs over the ranks that have one: -inf elsewhere
    m[I_RET] = torch.where(v[I_NRET] > 0, v[I_RET], torch.full_like(v[I_RET], -math.inf))
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return s, m


def replica_train(engine, replay, n_steps: int, chunk: int, every: int = 1024, group=None) -> List[Tuple]:
    """``n_steps`` gradient steps of this rank's learner (hipGraph chunks of
    ``chunk``), the replica metric vector all-reduced after every block of
    ``every`` steps (and after the last, partial block) when torch.distributed
    is initialised.  Returns the [(sum, max)] device tensors of every
    aggregation; ``summarise_aggregates`` reads them (a sync) once training is
    over."""
    on = _initialised()
    out = []
    done = 0
    every = max(1, int(every))
    t0 = time.perf_counter()
    while done < n_steps:
        k = min(every, n_steps - done)
        engine.train_graph(replay, k, chunk)
        done += k
        if on:  # wall_s: host time of the enqueues so far; mean_return: no episodes in a bench
            out.append(aggregate_device(metric_vector(engine, time.perf_counter() - t0), group))
    return out


class ReplicaAggregator:
    """``callback`` of ``SAC.run_vectorized_training_loop`` for replica
    training (sac/train_replicas.py): every ``every`` gradient steps of this
    rank's learner (and once more at ``finish``) the replica metric vector
    METRICS -- the engine's step counter, losses and alpha, this rank's wall
    time and the mean return of its last 100 episodes -- is all-reduced
    (sum and max) over the process group, on the device, without a host sync
    (RCCL orders the collectives after the training stream's work).  Without an
    initialised process group the rank's own vector is kept."""

    def __init__(self, engine, every: int = 1024, group=None):
        self.engine, self.group = engine, group
        self.every = max(1, int(every))
        self.next = self.every
        self.t0 = time.perf_counter()
        self.aggs: List[Tuple] = []
        self.last: dict = {}

    def _aggregate(self, st: dict) -> None:
        v = metric_vector(self.engine, time.perf_counter() - self.t0, st.get("avg_return", float("nan")),
                          steps=st.get("gradient_steps", 0))
        if _initialised():
            self.aggs.append(aggregate_device(v, self.group))
        else:
            m = v.clone()
            if m[I_NRET] <= 0:
                m[I_RET] = -math.inf
            self.aggs.append((v, m))

    def __call__(self, st: dict) -> None:
        self.last = st
        if st["gradient_steps"] >= self.next:
            self.next = (st["gradient_steps"] // self.every + 1) * self.every
            self._aggregate(st)

    def finish(self) -> dict:
        """The final aggregation (after the loop's last step) and its host view."""
        self._aggregate(self.last)
        import torch.distributed as dist

        world = dist.get_world_size(self.group) if _initialised() else 1
        return summarise_aggregates(self.aggs, world, self.every)


def summarise_aggregates(aggs, world: int, every: int) -> dict:
    """Host view of replica_train's aggregates (reads device memory)."""
    if not aggs:
        return {"every": every, "aggregations": 0}
    s, m = aggs[-1]
    s, m = s.tolist(), m.tolist()
    fin = lambda xs: [x if math.isfinite(x) else None for x in xs]  # noqa: E731  (JSON: no NaN)
    mean = [x / world for x in s]
    n_ret = s[I_NRET]
    # mean_return: over the ranks that have finished an episode
    mean[I_RET] = s[I_RET] / n_ret if n_ret > 0 else float("nan")
    if n_ret <= 0:
        s[I_RET] = float("nan")
    return {"every": every, "aggregations": len(aggs), "world": world, "fields": list(REPLICA_METRICS),
            "last_sum": fin(s), "last_mean": fin(mean), "last_max": fin(m)}


def timed_region(run, sync, device: Optional[torch.device] = None, group=None) -> float:
    """Wall time of ``run()`` bracketed by (barrier + ``sync()``) on both sides,
    MAX over ranks (the bench contract; single process when not initialised)."""
    import torch.distributed as dist

    on = _initialised()
    sync()
    if on:
        dist.barrier(group)
        sync()
    t0 = time.perf_counter()
    run()
    sync()
    if on:  # one process: the device is idle after the first sync (a second one only adds host latency)
        dist.barrier(group)
        sync()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if on:
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=group)
    return float(el.item())


def aggregate_throughput(steps: int, wall_s: float, group=None, device=None) -> float:
    """Whole-job steps/s: total steps of all replicas / slowest replica's time."""
    agg = aggregate_metrics([steps, wall_s], group, device)
    return agg["sum"][0] / agg["max"][1]
