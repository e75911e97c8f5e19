"""Multi-GPU layer on the CPU: independent-seed replicas, metric aggregation
over torch.distributed (gloo, world_size 2; the GPU job uses RCCL), and the
bench's whole-job throughput rule (total steps / slowest replica)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sac.replicas import METRICS, aggregate_metrics, aggregate_throughput, replica_seed, timed_region


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vals = [100.0 * (rank + 1), 2.0 + rank, 1.0 + rank, 2.0, -1.0 * rank, 0.5, 0.1, 10.0 * rank]
        agg = aggregate_metrics(vals)
        tput = aggregate_throughput(1000 * (rank + 1), 2.0 + rank)
        seeds = torch.tensor([replica_seed(42, rank)])
        gathered = [torch.zeros_like(seeds) for _ in range(world)]
        dist.all_gather(gathered, seeds)
        import time

        el = timed_region(lambda: time.sleep(0.05 + 0.25 * rank), lambda: None)
        out[rank] = (agg, tput, [int(g) for g in gathered], el)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_replica_aggregation_gloo(world):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert set(out.keys()) == set(range(world))
    for r in range(world):
        agg, tput, seeds, el = out[r]
        assert 0.29 <= el < 2.0                                # max over ranks: the slow rank's time
        assert agg["world"] == world
        assert agg["sum"][0] == pytest.approx(300.0)          # steps summed
        assert agg["max"][1] == pytest.approx(3.0)            # slowest wall time
        assert agg["mean"][2] == pytest.approx(1.5)           # losses averaged
        assert tput == pytest.approx(3000.0 / 3.0)            # total steps / slowest replica
        assert seeds == [42, 43]                              # distinct replica seeds
    assert len(METRICS) == 9 and METRICS[7] == "mean_return"
