"""bench.py's multi-GPU path on the CPU (SAC_BENCH_STUB=1: the engine is a
host stub, torch.distributed runs on gloo): ``python bench.py --gpus 2`` with
no torchrun environment starts its own two rank processes before any GPU
call, the ranks time the same region (barrier + max over ranks), all-reduce
the replica metric vector every --aggregate-every steps inside it, and rank 0
prints one JSON line with n_gpus 2 and parallelism replicas2.  A --gpus that
disagrees with a torchrun WORLD_SIZE fails loudly."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(SAC_BENCH_STUB="1", **kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_spawns_its_ranks_and_reports_replicas():
    p = _run(["--gpus", "2", "--steps", "40", "--warmup", "4", "--chunk", "8", "--aggregate-every", "16"], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "replicas2"
    assert line["steps"] == 40 and line["scaling"] == "weak"
    # whole-job throughput: both ranks' steps over the slowest rank's wall time
    # (rank 1's stub steps take 30 us, rank 0's 20 us: >= 40 x 30 us)
    assert line["value"] == pytest.approx(80 / (line["ms_per_step"] * 40 / 1e3), rel=1e-3)
    assert line["ms_per_step"] >= 0.030
    rm = line["replica_metrics"]
    assert rm["aggregations"] == 3 and rm["every"] == 16 and rm["world"] == 2  # 16 + 16 + 8 steps
    assert rm["fields"][0] == "steps"
    assert rm["last_sum"][0] == 2 * (4 + 40)  # each replica's step counter: warm-up + timed
    assert rm["last_max"][0] == 4 + 40
    assert rm["fields"][2] == "q1_loss" and rm["fields"][7] == "mean_return"
    assert rm["last_mean"][2] == pytest.approx(1.0)  # the stub's L_Q1 on both ranks
    assert rm["last_max"][1] > 0  # wall_s: the slower rank's time so far
    assert rm["last_sum"][7] is None  # mean_return: no episodes in a bench (NaN -> null)


def test_bench_single_gpu_runs_in_process():
    p = _run(["--steps", "10", "--warmup", "2"], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "replicas1"
    assert "replica_metrics" not in line


def test_bench_rejects_gpus_world_size_mismatch():
    p = _run(["--gpus", "3", "--steps", "4"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in p.stderr
