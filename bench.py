"""SAC gradient steps/s + replay-sample GB/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c4w|c1]
                    [--precision bf16|fp32] [--no-cpu-baseline]

A "step" is one full SAC gradient step (device sample + gather, target, both
critic updates, actor update, alpha update, Polyak) on a full synthetic 1e6-row
replay buffer resident in HBM, replayed from hipGraphs.  For N > 1 each rank is
an independent-seed replica on its own GPU (replicas only: the step does not
shard), training through sac.replicas.replica_train, which all-reduces the
replica metric vector over RCCL every --aggregate-every steps inside the timed
region; value = total steps of all ranks / max wall time.  The ranks come
from torchrun (WORLD_SIZE set; it must equal --gpus) or, when --gpus N > 1 is
given without it, from this script itself (launch_ranks: one child process
per GPU, started before anything touches the GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "soft-actor-critic_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    # BASELINE.json configs; obs, act, hidden, buffer, batch
    "c1": dict(obs=4, act=1, hidden=[64, 64], capacity=10_000, batch=64, name="InvertedPendulum-v5"),
    "c2": dict(obs=24, act=4, hidden=[256, 256], capacity=1_000_000, batch=256, name="BipedalWalker-v3"),
    "c3": dict(obs=24, act=4, hidden=[256, 256], capacity=1_000_000, batch=4096, name="BipedalWalker-v3"),
    "c4": dict(obs=32, act=2, hidden=[256, 256], capacity=1_000_000, batch=256, name="DonkeyVae-v0-level-0"),
    "c4w": dict(obs=216, act=2, hidden=[256, 256], capacity=1_000_000, batch=256, name="DonkeyVae-v0 (obs 216)"),
}
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # MI355X_MICROARCH.md: dense MFMA peaks
PEAK_HBM_GBS = 8000.0


def gemm_flops(obs, act, hidden, B):
    """Algorithmic GEMM FLOPs per launch of each phase kernel."""
    qd = [obs + act] + hidden + [1]
    pd = [obs] + hidden + [2 * act]
    G = lambda d: sum(d[i] * d[i + 1] for i in range(len(d) - 1))  # noqa: E731
    Gq, Gp = G(qd), G(pd)
    Gq1, Gp1 = Gq - qd[0] * qd[1], Gp - pd[0] * pd[1]
    A = 2 * B * (2 * Gp + 4 * Gq + 2 * Gq1)      # pi fwd (s,s'), 2 target + 2 critic fwd, critic dX
    Bk = 2 * B * (2 * Gq)                         # critic dW
    C = 2 * B * (4 * Gq + Gp1)                    # critic fwd on (s,a~), critic dX down to a~, pi dX
    D = 2 * B * Gp                                 # pi dW
    total_survey = 2 * B * (3 * Gp + Gp1 + 10 * Gq + 2 * Gq1)  # SURVEY §8d F_alg
    return [A, Bk, C, D], total_survey, Gq, Gp


def soa_copy(rb):
    """The same rows in a struct-of-arrays replay (layout comparison leg of the sweep)."""
    from sac.replay_buffer import ReplayBuffer

    soa = ReplayBuffer(rb.capacity, device=rb.device, obs_dim=rb.obs_dim, act_dim=rb.act_dim, layout="soa")
    soa.push_batch(rb.obs, rb.act, rb.rew, rb.next_obs, rb.done)
    torch.cuda.synchronize()
    return soa


def synthetic_replay(rb, cap, obs, act, seed):
    """s~N(0,1), a~U(-1,1), r~N(0,1), d~Bernoulli(.01), s' = next row's s."""
    rng = np.random.default_rng(seed)
    chunk = 250_000
    s_all = rng.standard_normal((cap + 1, obs), dtype=np.float32)
    for i in range(0, cap, chunk):
        n = min(chunk, cap - i)
        s = s_all[i:i + n]
        s2 = s_all[i + 1:i + 1 + n]
        a = rng.uniform(-1, 1, (n, act)).astype(np.float32)
        r = rng.standard_normal(n, dtype=np.float32)
        d = (rng.random(n) < 0.01).astype(np.float32)
        rb.push_batch(s, a, r, s2, d)
    torch.cuda.synchronize()


def build_engine(cfgname, precision, seed, device, capacity=None, layout=None):
    """Engine + synthetic replay of a CONFIGS entry.  ``layout``: kernel layout
    overrides for the tests (sac.engine.SacEngine); None = the engine's choice."""
    from sac.engine import SacEngine
    from sac.models import PolicyNetwork, QNetwork
    from sac.replay_buffer import ReplayBuffer

    c = dict(CONFIGS[cfgname])
    if capacity:
        c["capacity"] = capacity
    pi = PolicyNetwork(c["obs"], c["act"], c["hidden"], seed=seed).to(device)
    q1 = QNetwork(c["obs"], c["act"], c["hidden"], seed=seed).to(device)
    q2 = QNetwork(c["obs"], c["act"], c["hidden"], seed=seed + 1).to(device)
    import copy

    q1t, q2t = copy.deepcopy(q1), copy.deepcopy(q2)
    # notebooks/configs/bipedal_walker.yaml:4-38 with auto_entropy_tuning on
    eng = SacEngine(pi, q1, q2, q1t, q2t, batch_size=c["batch"], gamma=0.99, tau=0.005, actor_lr=3e-4,
                    critic_lr=3e-4, alpha_lr=3e-4, alpha=0.1, auto_entropy_tuning=True, device=device,
                    precision=precision, seed=seed, layout=layout)
    rb = ReplayBuffer(c["capacity"], device=device, obs_dim=c["obs"], act_dim=c["act"])
    synthetic_replay(rb, c["capacity"], c["obs"], c["act"], seed)
    return eng, rb, c


def prewarm(rb, device, seconds):
    """Device clock pre-warm: `seconds` of back-to-back replay gathers (B = 65,536
    uniform rows of the synthetic buffer into scratch tensors) before the warm-up
    steps.  No SAC step runs and no learner state is touched.  Measured with
    the driver's short form (--steps 20 --warmup 5; one graph replay timed): it
    read 16.0K steps/s, every phase kernel ~1.8 us longer than in a 2,000-step
    run (18.3K), because the graph capture's host work left the device idle
    right before the timed region.  Capturing first: 17.4K; with this pre-warm
    as well: 17.6K (profiles/r02_bench_short_form.txt)."""
    if seconds <= 0:
        return
    from sac import _engine as E
    import ctypes

    lib = E.load_library()
    st = E.stream_handle(device)
    B = 65536
    f = dict(dtype=torch.float32, device=device)
    outs = [torch.empty(B, rb.obs_dim, **f), torch.empty(B, rb.act_dim, **f), torch.empty(B, **f),
            torch.empty(B, rb.obs_dim, **f), torch.empty(B, **f)]
    ptrs = [E.ptr(t) for t in outs]
    ridx = torch.randint(0, len(rb), (B,), dtype=torch.int32, device=device)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(50):
            E.check(lib.sac_replay_gather(ctypes.byref(rb.desc), E.ptr(ridx), B, *ptrs, st))
        torch.cuda.synchronize()


def gather_sweep(rb, device, sizes=(256, 4096, 65536, 1_048_576), reps=20):
    """Standalone replay sample + gather (SURVEY §8d roofline leg), two forms:
      sample_gather: the device sampler's B distinct rows gathered in ONE kernel
                     (sac_replay_sample_gather), for B <= len(rb);
      gather:        sac_replay_gather of B uniform rows drawn WITH replacement
                     (torch.randint, outside the timed loop) -- the bandwidth leg,
                     which also runs B = 1,048,576 > the 1e6-row buffer.
    Returns {form: {B: GB/s}} with GB/s = B_gather / kernel time, B_gather =
    4 B (2 obs + act + 2) bytes read (the gather writes as many
    again), plus the per-launch ms of each point: `reps` back-to-back launches
    timed with hipEvents on the launch stream, and (as "ms_graph") the same
    launches captured in one hipGraph and timed around its replay (measured:
    within ~10% of the eager figure; the graph form is the slower one at
    B = 65,536)."""
    from sac import _engine as E
    import ctypes

    lib = E.load_library()
    W = 2 * rb.obs_dim + rb.act_dim + 2
    st = E.stream_handle(device)
    desc = rb.desc
    out = {"sample_gather": {}, "gather": {}, "ms": {}, "ms_graph": {}}
    f = dict(dtype=torch.float32, device=device)
    for B in sizes:
        s, a, r, s2, d = (torch.empty(B, rb.obs_dim, **f), torch.empty(B, rb.act_dim, **f), torch.empty(B, **f),
                          torch.empty(B, rb.obs_dim, **f), torch.empty(B, **f))
        ptrs = [E.ptr(t) for t in (s, a, r, s2, d)]
        ridx = torch.randint(0, len(rb), (B,), dtype=torch.int32, device=device,
                             generator=torch.Generator(device=device).manual_seed(B))
        forms = {"gather": lambda k, st: E.check(lib.sac_replay_gather(ctypes.byref(desc), E.ptr(ridx), B, *ptrs, st))}
        if B <= len(rb):
            forms["sample_gather"] = lambda k, st: E.check(lib.sac_replay_sample_gather(
                ctypes.byref(desc), B, 7, k, None, *ptrs, st))
        for form, once in forms.items():
            for k in range(3):
                once(k, st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(reps):
                once(k, st)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            out[form][str(B)] = round(B * W * 4 / (ms * 1e-3) / 1e9, 3)
            out["ms"][f"{form}/{B}"] = round(ms, 5)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                cst = E.stream_handle(device)  # the capture stream
                for k in range(reps):
                    once(k, cst)
            g.replay()
            torch.cuda.synchronize()
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            del g
            out["ms_graph"][f"{form}/{B}"] = round(e0.elapsed_time(e1) / reps, 5)
    return out


def bf16_deviation(cfgname, seed, device, steps=3):
    """The bf16 perf mode's loss deviation: fp32 and bf16 engines from the same
    init (bench.build_engine seeding) fed the same injected indices and eps for
    `steps` steps; max over steps of |L_bf16 - L_fp32| / max(|L_fp32|, floor)
    per loss (floor 1e-3; L_pi: mean|y| of the step, as tests/test_gpu_parity.py).
    The fp32 engine is the parity mode tests/ pin against the oracle at 1e-4."""
    c = CONFIGS[cfgname]
    engs = {p: build_engine(cfgname, p, seed, device, capacity=max(4096, c["batch"] * 2)) for p in ("fp32", "bf16")}
    B, A = c["batch"], c["act"]
    g = np.random.default_rng(123)
    dev = [0.0] * 4
    for _ in range(steps):
        idx = torch.from_numpy(g.choice(len(engs["fp32"][1]), size=(1, B), replace=False).astype(np.int32))
        eps = torch.from_numpy(g.standard_normal((1, 2, B, A)).astype(np.float32))
        res = {}
        for p, (eng, rb, _) in engs.items():
            eng.train(rb, 1, indices=idx, eps=eps)
            res[p] = (eng.losses(), float(eng.last_targets().abs().mean()))
        (lf, ym), (lb, _) = res["fp32"], res["bf16"]
        for i in range(4):
            if np.isnan(lf[i]):
                continue
            floor = ym if i == 2 else 1e-3
            dev[i] = max(dev[i], abs(lb[i] - lf[i]) / max(abs(lf[i]), floor))
    return {"loss_rel_dev_vs_fp32": [round(x, 7) for x in dev], "steps": steps,
            "losses": ["L_Q1", "L_Q2", "L_pi (floor mean|y|)", "L_alpha"]}


def short_kernel(name):
    """The phase-kernel family of a kernel name (tools/pmc_summary.short: the
    split and stage variants count under their phase's family)."""
    for k in ("sac_target_critic", "sac_critic_update", "sac_actor_update", "sac_actor", "sac_wide_stage"):
        if k in name:
            return k
    return name


def pmc_traffic(kernel, config, precision):
    """HBM-side bytes per launch of `kernel` from the newest committed PMC
    summary for this (config, precision) (profiles/<round>_pmc*.json, written
    by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench), or (None, None)."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("config", "c2") != config or d.get("precision", "bf16") != precision:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k:
            return k["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(cfgname, seconds=5.0):
    """The reference CPU path on the host: the oracle (numpy restatement of the
    reference step, incl. its deque + random.sample replay over the full
    buffer) timed per BASELINE.md §4 -- BLAS threads 1 and T (T = the host's
    CPU share: OMP_NUM_THREADS, else os.cpu_count()), full training_step()s and
    update-only steps (batch sampled outside the timed loop), `seconds` each.
    value = the faster full-step leg; every leg is listed."""
    from threadpoolctl import threadpool_limits

    from oracle import sac_oracle as O

    c = CONFIGS[cfgname]
    rng = np.random.default_rng(0)
    cap = c["capacity"]
    buf = O.ReplayDeque(cap)
    s_all = rng.standard_normal((cap + 1, c["obs"]), dtype=np.float32)
    a_all = rng.uniform(-1, 1, (cap, c["act"])).astype(np.float32)
    r_all = rng.standard_normal(cap, dtype=np.float32)
    d_all = rng.random(cap) < 0.01
    for i in range(cap):
        buf.push(s_all[i], a_all[i], float(r_all[i]), s_all[i + 1], bool(d_all[i]))

    def mlp(dims, seed):
        g = np.random.default_rng(seed)
        W, b = [], []
        for i in range(len(dims) - 1):
            lim = np.sqrt(6.0 / (dims[i] + dims[i + 1]))
            W.append(g.uniform(-lim, lim, (dims[i + 1], dims[i])).astype(np.float32))
            b.append(np.zeros(dims[i + 1], np.float32))
        return O.MLP(W, b)

    hp = O.SacHyper(auto_entropy_tuning=True)
    O_, A_ = c["obs"], c["act"]
    st = O.SacState.fresh(mlp([O_] + c["hidden"] + [2 * A_], 0), mlp([O_ + A_] + c["hidden"] + [1], 1),
                          mlp([O_ + A_] + c["hidden"] + [1], 2), hp, A_)
    B = c["batch"]
    erng = np.random.default_rng(1)
    nthr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    fixed = O.sample_batch(buf, B)
    legs = []
    for threads in (1, nthr):
        for kind in ("full", "update_only"):
            n = 0
            with threadpool_limits(limits=threads):
                t0 = time.perf_counter()
                while True:
                    b = O.sample_batch(buf, B) if kind == "full" else fixed
                    O.training_step(st, hp, b, erng.standard_normal((B, A_), dtype=np.float32),
                                    erng.standard_normal((B, A_), dtype=np.float32))
                    n += 1
                    el = time.perf_counter() - t0
                    if el >= seconds:
                        break
            legs.append({"threads": threads, "kind": kind, "steps_per_s": round(n / el, 3), "steps": n,
                         "seconds": round(el, 2)})
    full = max((l for l in legs if l["kind"] == "full"), key=lambda l: l["steps_per_s"])
    return {"value": full["steps_per_s"], "unit": "gradient steps/s", "cores": full["threads"], "kind": "port",
            "sample": f"full training_step()s (deque+random.sample over {cap} rows, B={B}) and update-only steps, "
                      f"numpy fp32, BLAS threads 1 and {nthr} (host CPU share), {seconds:.0f}s per leg",
            "host_threads": nthr, "legs": legs}


class _StubEngine:
    """SAC_BENCH_STUB=1 (tests/test_bench_ranks.py, CPU only): the rank and
    launcher logic of this file without the HIP engine -- a learner whose
    graph-replayed steps sleep 20 us (+10 us per rank) on the host and whose
    state tensors are CPU tensors."""

    fused = 0

    def __init__(self, batch, rank):
        self.batch, self.rank, self.steps_done = batch, rank, 0
        self.rng_step = torch.zeros(1, dtype=torch.int64)
        self.stats = torch.tensor([1.0, 2.0, -0.5, 0.1] + [0.0] * (2 * batch), dtype=torch.float32)
        self.alpha_state = torch.tensor([-2.3, 0.1, 0.0, 0.0], dtype=torch.float64)

    def train_graph(self, rb, n, chunk):
        time.sleep(n * (20 + 10 * self.rank) * 1e-6)
        self.rng_step += n
        self.steps_done += n

    def check(self):
        pass

    def losses(self):
        return self.stats[:4].double().tolist()


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` (N > 1) without torchrun: start one rank process per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free
    MASTER_PORT), each running this file with the same arguments.  This
    process never touches the GPU (no torch.cuda call before or after), so the
    ranks start clean; it waits for them and returns the first non-zero exit
    status (stopping the other ranks then, so none waits at a barrier for a
    dead peer), else 0.  Rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # our own children, by handle
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"],
                    help="headline arithmetic; fp32 is the reference's (bf16 is also timed unless --no-bf16)")
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--aggregate-every", type=int, default=1024,
                    help="replicas (N > 1): gradient steps between the RCCL metric all-reduces (SURVEY §8e)")
    ap.add_argument("--prewarm", type=float, default=0.3,
                    help="seconds of replay gathers before the warm-up steps (device clocks; no SAC step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 (B = 4096) legs of the c2 line")
    ap.add_argument("--layout", default="", help="A/B runs only: kernel layout overrides of the headline leg, "
                    "'key=value,...' over sac._engine.LAYOUT_KEYS (e.g. layout=rows,upd_parts=4); default: "
                    "the engine's own choice")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(world_env or 1)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (torchrun --nproc-per-node must "
                         f"equal --gpus)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    run_rank(args, world, rank, local)


def run_rank(args, world, rank, local):
    stub = os.environ.get("SAC_BENCH_STUB") == "1"
    if stub:
        device = torch.device("cpu")
        sync = lambda: None  # noqa: E731
        args.no_sweep = args.no_bf16 = args.no_cpu_baseline = args.no_c3 = True
    else:
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
        sync = torch.cuda.synchronize
    dist = None
    if world > 1:
        import torch.distributed as dist

        if stub:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from sac.replicas import replica_seed, replica_train, summarise_aggregates, timed_region

    seed = replica_seed(0, rank)
    # graph chunk <= the timed steps, so a short driver run is graph-replayed too
    chunk = max(1, min(args.chunk, args.steps))
    every = args.aggregate_every

    layout = {}
    for kv in filter(None, args.layout.split(",")):
        k, v = kv.split("=")
        layout[k] = v if k == "layout" else int(v)

    def timed(precision, cfgname, steps=None, warmup=None):
        steps = args.steps if steps is None else steps
        warmup = args.warmup if warmup is None else warmup
        if stub:
            c = dict(CONFIGS[cfgname])
            eng, rb = _StubEngine(c["batch"], rank), None
        else:
            eng, rb, c = build_engine(cfgname, precision, seed, device, layout=layout or None)
            # capture (+ upload) the chunk graph first (runs no step): its host-side work
            # would otherwise leave the device idle between the warm-up and the timed region
            eng.train_graph(rb, 0, chunk)
            prewarm(rb, device, args.prewarm)
        eng.train_graph(rb, warmup, chunk)
        aggs = []
        if dist:  # replicas: the metric all-reduce every `every` steps runs inside the timed region
            el = timed_region(lambda: aggs.extend(replica_train(eng, rb, steps, chunk, every)), sync, device)
        else:
            el = timed_region(lambda: eng.train_graph(rb, steps, chunk), sync, device)
        eng.check()  # in-launch hand-offs all completed (raises HandoffTimeout otherwise)
        ls = eng.losses()
        if not all(np.isfinite(ls[:3])):
            raise SystemExit(f"non-finite losses after benchmark ({precision}): {ls}")
        return eng, rb, c, el, ls, aggs

    eng, rb, c, elapsed, losses, aggs = timed(args.precision, args.config)
    total_steps = args.steps * world
    replica = summarise_aggregates(aggs, world, every) if dist else None
    sps = total_steps / elapsed
    line = {
        "metric": "SAC gradient steps/sec + replay-sample GB/s, BipedalWalker batch=256",
        "value": round(sps, 2),
        "unit": "gradient steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (numpy default_rng, SURVEY §8d), random-init reference-seeded weights",
        "config": {"workload": f"{args.config}: {c['name']} obs={c['obs']} act={c['act']} "
                               f"2x{c['hidden']} MLPs, buffer={c['capacity']}, batch={c['batch']}, "
                               f"auto-alpha, device sampler, {args.precision} arithmetic",
                   "global_batch": c["batch"] * world, "parallelism": f"replicas{world}",
                   "graph_chunk": chunk, "device_prewarm_s": args.prewarm},
    }
    if layout:
        line["config"]["layout_override"] = layout  # an A/B run, not the engine's own choice
    if stub:
        line["stub"] = "SAC_BENCH_STUB=1: rank/launcher logic only, no engine"
    else:
        line.update(measure_phases(args, eng, rb, c, elapsed, sps / world))
        line["losses_last"] = [round(x, 6) for x in losses]
    if replica is not None:
        line["replica_metrics"] = replica
    if rank == 0 and not stub:
        if not args.no_sweep:
            line.update(sweep_fields(rb, c, device))
        if not args.no_bf16 and args.precision == "fp32" and world == 1:  # single-process leg: no barriers
            eb, rbb, _, elb, lsb, _ = timed("bf16", args.config)
            line["value_bf16"] = round(total_steps / elb, 2)
            line["ms_per_step_bf16"] = round(elb / args.steps * 1e3, 5)
            line["bf16_parity"] = bf16_deviation(args.config, seed, device)
            del eb, rbb
        if not args.no_c3 and args.config == "c2" and world == 1:
            line.update(c3_legs(args, timed))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def mfma_busy(kernel, config, precision):
    """Counter-based MFMA-busy fraction of `kernel` (SQ_VALU_MFMA_BUSY_CYCLES over
    the launch's SIMD cycles) from the newest committed profiles/<round>_mfma_busy.json
    (tools/sq_summary.py), or (None, None)."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_mfma_busy.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        for key in (f"{config}_{precision}/{kernel}", f"sq_{config}_{precision}/{kernel}"):
            k = d.get("kernels", {}).get(key)
            if k and "mfma_busy_frac" in k:
                return k["mfma_busy_frac"], os.path.relpath(path, ROOT)
    return None, None


def measure_phases(args, eng, rb, c, elapsed, sps_one):
    """Per-phase device time (hipEvents on the launch stream) and the roofline
    of the dominant kernel.  Each interval also holds the cost of the event
    after it; the timed region ran the same launches from hipGraphs with no
    events.  The per-launch event cost = (sum of the intervals of one step -
    the event-free step time) / launches per step; interval - that cost = the
    kernel's own duration (the figure rocprofv3 --kernel-trace reports:
    profiles/<round>_kernel_stats*.csv)."""
    from sac import _engine as E

    tp = eng.time_phases(rb, 100)
    phase_ms, empty_ms = tp[:4], tp[4]
    step_ms = elapsed / args.steps * 1e3
    # launches per step of each phase (the stage path runs several per phase):
    # each launch's interval also holds one event
    nl = [n if x > 0 else 0 for n, x in zip(eng.phase_launches, phase_ms)]
    ev_cost = max((sum(phase_ms) - step_ms) / max(sum(nl), 1), 0.0)
    kern_ms = [x - ev_cost * n if x > 0 else 0.0 for x, n in zip(phase_ms, nl)]
    flops, f_total, _, _ = gemm_flops(c["obs"], c["act"], c["hidden"], c["batch"])
    dom = int(np.argmax(phase_ms))
    lib = E.load_library()
    kname = lib.sac_phase_kernel_name(dom).decode()
    traffic, traffic_src = pmc_traffic(kname, args.config, args.precision)
    achieved = flops[dom] / (kern_ms[dom] * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]
    # phases A and C (the two heaviest launches) side by side: FLOP fraction of
    # the dtype's dense peak over the event-timed launch, and the SQ counters'
    # MFMA-busy fraction of the same kernel (committed counter file)
    phases = {}
    for i, ph in ((0, "A"), (2, "C")):
        if kern_ms[i] <= 0:
            continue
        kn = lib.sac_phase_kernel_name(i).decode()
        busy, busy_src = mfma_busy(short_kernel(kn), args.config, args.precision)
        a = flops[i] / (kern_ms[i] * 1e-3) / 1e12
        phases[ph] = {"kernel": kn, "flops_per_launch": flops[i], "avg_launch_ms": round(kern_ms[i], 5),
                      "achieved": round(a, 3), "frac": round(a / peak, 5), "counter_mfma_busy_frac": busy,
                      "counter_source": busy_src}
    W = 2 * c["obs"] + c["act"] + 2
    return {
        "replay_sample_GBps_in_step": round(sps_one * c["batch"] * W * 4 / 1e9, 4),
        "phase_ms": [round(x, 5) for x in kern_ms],
        "phase_event_interval_ms": [round(x, 5) for x in phase_ms],
        "event_cost_ms": round(ev_cost, 5),
        "phase_launches_per_step": nl,
        "empty_kernel_event_interval_ms": round(empty_ms, 5),
        "step_gemm_flops_survey": f_total,
        "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 5), "traffic": traffic,
                     "traffic_source": traffic_src, "flops_per_launch": flops[dom],
                     "avg_launch_ms": round(kern_ms[dom], 5),
                     "timing": "hipEvents after every launch on the launch stream over 100 steps; "
                               "avg_launch_ms = mean interval of this kernel's launches minus the per-launch "
                               "event cost (event intervals of a step - event-free graph step time, per launch)"},
        "roofline_phases": phases,
        "step_roofline": {"achieved_TFLOPs": round(f_total * sps_one / 1e12, 3), "peak": peak,
                          "frac": round(f_total * sps_one / 1e12 / peak, 5),
                          "note": "SURVEY F_alg per step x steps/s of one learner"},
    }


def c3_legs(args, timed):
    """C3 (BASELINE configs[2]: B = 4096, the MFMA-bound regime) on the same
    line, so the driver times it: fp32 and bf16 steps/s, graph-replayed like
    the headline, with the step's fraction of the dtype's dense MFMA peak
    (SURVEY F_alg per step x steps/s).  C3 steps are ~4-8x longer than C2's,
    so the timed steps are scaled down (at least 20) to keep the run short."""
    out = {}
    steps, warmup = max(20, args.steps // 8), max(5, args.warmup // 8)
    f_total = gemm_flops(24, 4, [256, 256], 4096)[1]
    for prec in ("fp32", "bf16"):
        eng, rb, c, el, ls, _ = timed(prec, "c3", steps, warmup)
        sps = steps / el
        key = "value_c3" if prec == "fp32" else "value_c3_bf16"
        out[key] = round(sps, 2)
        out[key + "_detail"] = {"steps": steps, "ms_per_step": round(el / steps * 1e3, 5),
                                "mfma_frac": round(f_total * sps / 1e12 / PEAK_TFLOPS[prec], 5),
                                "peak_TFLOPs": PEAK_TFLOPS[prec], "losses_last": [round(x, 6) for x in ls]}
        del eng, rb
        torch.cuda.empty_cache()
    return out


def copy_ceiling(nbytes, device, reps=20):
    """Same-box ceiling for the gather leg: plain device
    copies of `nbytes` (nbytes read + nbytes written per launch, contiguous),
    timed like gather_sweep.  Returns {form: GB/s read + write}."""
    src = torch.rand(nbytes // 4, device=device)
    dst = torch.empty_like(src)
    out = {}
    for name, fn in (("copy_", lambda: dst.copy_(src)), ("mul_out", lambda: torch.mul(src, 1.0, out=dst))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9, 1)
    del src, dst
    return out


def time_gather(rb, idx_sets, B, device, reps=20):
    """ms per sac_replay_gather launch of B rows, rep k reading idx_sets[k % len]
    (hipEvents around `reps` back-to-back launches on the launch stream)."""
    from sac import _engine as E
    import ctypes

    lib = E.load_library()
    st = E.stream_handle(device)
    desc = rb.desc
    f = dict(dtype=torch.float32, device=device)
    outs = (torch.empty(B, rb.obs_dim, **f), torch.empty(B, rb.act_dim, **f), torch.empty(B, **f),
            torch.empty(B, rb.obs_dim, **f), torch.empty(B, **f))
    ptrs = [E.ptr(t) for t in outs]
    once = lambda ix: E.check(lib.sac_replay_gather(ctypes.byref(desc), E.ptr(ix), B, *ptrs, st))  # noqa: E731
    for k in range(3):
        once(idx_sets[k % len(idx_sets)])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        once(idx_sets[k % len(idx_sets)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def gather_ceilings(rb, c, device, B=1_048_576, big_rows=4_000_000):
    """like-for-like ceilings of the gather leg, the SAME
    kernel (replay_gather_records_kernel) on the same kind of table:
      * same 1e6-row table, its rows read in table order (logical i % size) --
        the streaming form of the random-row gather, same MALL residency;
      * a 4e6-row table (1 GB of records, past the 256 MiB Infinity Cache):
        random rows (4 independent draws rotating over the reps, ~1 GB touched)
        and rows in table order (4 disjoint 1M-row windows rotating: every rep
        streams a fresh 256 MB), so the HBM fraction is not flattered by on-die
        hits.  GB/s = B_gather (SURVEY §8d bytes read) / launch time."""
    from sac.replay_buffer import ReplayBuffer

    W = 2 * c["obs"] + c["act"] + 2
    gbs = lambda ms: round(B * W * 4 / (ms * 1e-3) / 1e9, 3)  # noqa: E731
    i32 = dict(dtype=torch.int32, device=device)
    seq = [(torch.arange(B, device=device, dtype=torch.int64) % len(rb)).to(torch.int32)]
    out = {"B": B, "same_table_rows_in_order_GBps": gbs(time_gather(rb, seq, B, device))}
    big = ReplayBuffer(big_rows, device=device, obs_dim=c["obs"], act_dim=c["act"])
    chunk = 500_000
    for i in range(0, big_rows, chunk):
        n = min(chunk, big_rows - i)
        g = torch.Generator(device=device).manual_seed(i)
        big.push_batch(torch.randn(n, c["obs"], device=device, generator=g),
                       torch.rand(n, c["act"], device=device, generator=g) * 2 - 1,
                       torch.randn(n, device=device, generator=g),
                       torch.randn(n, c["obs"], device=device, generator=g),
                       torch.rand(n, device=device, generator=g) < 0.01)
    torch.cuda.synchronize()
    rnd = [torch.randint(0, big_rows, (B,), generator=torch.Generator(device=device).manual_seed(k), **i32)
           for k in range(4)]
    win = [torch.arange(k * B, (k + 1) * B, **i32) % big_rows for k in range(4)]
    r_ms, s_ms = time_gather(big, rnd, B, device), time_gather(big, win, B, device)
    out["big_table"] = {"rows": big_rows, "table_MB": round(big_rows * big.row_stride * 4 / 1e6, 1),
                        "random_GBps": gbs(r_ms), "rows_in_order_GBps": gbs(s_ms),
                        "random_ms": round(r_ms, 5), "rows_in_order_ms": round(s_ms, 5),
                        "random_frac_of_hbm_peak": round(gbs(r_ms) / PEAK_HBM_GBS, 5),
                        "random_frac_of_rows_in_order": round(s_ms / r_ms, 4)}
    del big, rnd, win
    torch.cuda.empty_cache()
    return out


def sweep_fields(rb, c, device):
    sweep = gather_sweep(rb, device)
    sweep_soa = gather_sweep(soa_copy(rb), device, sizes=(65536, 1_048_576))
    W = 2 * c["obs"] + c["act"] + 2
    line = {}
    line["replay_sample_GBps_sweep"] = sweep["sample_gather"]
    line["replay_gather_GBps_sweep"] = sweep["gather"]
    line["replay_layout"] = f"transition records, row stride {rb.row_stride} floats"
    line["replay_gather_GBps_sweep_soa_layout"] = sweep_soa["gather"]
    line["replay_gather_ms_per_launch"] = {"eager": sweep["ms"], "graph": sweep["ms_graph"]}
    bmax = max(int(b) for b in sweep["gather"])
    ms = sweep["ms"][f"gather/{bmax}"]
    gk = ("replay_gather_records_kernel" if rb.layout == "records" and rb.row_stride in (16, 32, 64, 128, 256)
          and c["obs"] % 4 == 0 and c["act"] % 4 == 0 else "replay_gather_kernel")
    gtr, gsrc = pmc_traffic(gk, "gather", "fp32")
    line["roofline_gather"] = {
        "bound": "hbm", "kernel": gk, "batch": bmax,
        "achieved": sweep["gather"][str(bmax)], "peak": PEAK_HBM_GBS, "unit": "GB/s",
        "frac": round(sweep["gather"][str(bmax)] / PEAK_HBM_GBS, 5), "traffic": gtr,
        "traffic_kind": "L2 fabric bytes (PMC FETCH_SIZE x2 + WRITE_SIZE): the 256 MB record table nearly fits "
                        "the 256 MiB Infinity Cache, so part of FETCH is served on-die, not by HBM",
        "achieved_read_write": round(2 * sweep["gather"][str(bmax)], 3),
        "frac_read_write": round(2 * sweep["gather"][str(bmax)] / PEAK_HBM_GBS, 5),
        "traffic_source": gsrc, "bytes_per_launch": bmax * W * 4, "avg_launch_ms": ms,
        "copy_ceiling_GBps_read_write": None, "frac_of_copy_ceiling": None,
        "note": "B_gather = 4 B (2 obs + act + 2) bytes read per launch (SURVEY §8d); the kernel writes "
                "as many again (the minibatch it returns), counted in achieved_read_write; reads exceed "
                "B_gather by the record padding (2O+A+2 floats stored in whole 128-B lines); rows uniform "
                "with replacement over the 1e6-row buffer"}
    cc = copy_ceiling(bmax * W * 4, device)
    rg = line["roofline_gather"]
    rg["copy_ceiling_GBps_read_write"] = max(cc.values())
    rg["copy_ceiling_forms"] = cc
    rg["frac_of_copy_ceiling"] = round(rg["achieved_read_write"] / max(cc.values()), 4)
    gc = gather_ceilings(rb, c, device, B=bmax)
    rg["same_table_rows_in_order_GBps"] = gc["same_table_rows_in_order_GBps"]
    rg["frac_of_rows_in_order"] = round(rg["achieved"] / gc["same_table_rows_in_order_GBps"], 4)
    rg["big_table"] = gc["big_table"]
    return line


if __name__ == "__main__":
    main()
