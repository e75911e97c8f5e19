"""SAC gradient steps/s + replay-sample GB/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c4w|c1]
                    [--precision bf16|fp32] [--no-cpu-baseline]

A "step" is one full SAC gradient step (device sample + gather, target, both
critic updates, actor update, alpha update, Polyak) on a full synthetic 1e6-row
replay buffer resident in HBM, replayed from hipGraphs.  For N > 1 (torchrun),
each rank is an independent-seed replica on its own GPU (replicas only: the
step does not shard); value = total steps of all ranks / max wall time.
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


def build_engine(cfgname, precision, seed, device):
    from sac.engine import SacEngine
    from sac.models import PolicyNetwork, QNetwork
    from sac.replay_buffer import ReplayBuffer

    c = CONFIGS[cfgname]
    pi = PolicyNetwork(c["obs"], c["act"], c["hidden"], seed=seed).to(device)
    q1 = QNetwork(c["obs"], c["act"], c["hidden"], seed=seed).to(device)
    q2 = QNetwork(c["obs"], c["act"], c["hidden"], seed=seed + 1).to(device)
    import copy

    q1t, q2t = copy.deepcopy(q1), copy.deepcopy(q2)
    # notebooks/configs/bipedal_walker.yaml:4-38 with auto_entropy_tuning on
    eng = SacEngine(pi, q1, q2, q1t, q2t, batch_size=c["batch"], gamma=0.99, tau=0.005, actor_lr=3e-4,
                    critic_lr=3e-4, alpha_lr=3e-4, alpha=0.1, auto_entropy_tuning=True, device=device,
                    precision=precision, seed=seed)
    rb = ReplayBuffer(c["capacity"], device=device, obs_dim=c["obs"], act_dim=c["act"])
    synthetic_replay(rb, c["capacity"], c["obs"], c["act"], seed)
    return eng, rb, c


def gather_sweep(rb, device, sizes=(256, 4096, 65536, 1_048_576), reps=20):
    """Standalone device sampler + SoA gather: GB/s of (s,a,r,s',d) delivered."""
    from sac import _engine as E
    import ctypes

    lib = E.load_library()
    out = {}
    W = 2 * rb.obs_dim + rb.act_dim + 2
    for B in sizes:
        if B > len(rb):
            continue
        idx = torch.empty(B, dtype=torch.int32, device=device)
        f = dict(dtype=torch.float32, device=device)
        s, a, r, s2, d = (torch.empty(B, rb.obs_dim, **f), torch.empty(B, rb.act_dim, **f), torch.empty(B, **f),
                          torch.empty(B, rb.obs_dim, **f), torch.empty(B, **f))
        st = E.stream_handle(device)
        desc = rb.desc

        def once(k):
            E.check(lib.sac_replay_sample_indices(ctypes.byref(desc), B, 7, k, E.ptr(idx), st))
            E.check(lib.sac_replay_gather(ctypes.byref(desc), E.ptr(idx), B, E.ptr(s), E.ptr(a), E.ptr(r),
                                          E.ptr(s2), E.ptr(d), st))

        for k in range(3):
            once(k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(reps):
            once(k)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[str(B)] = round(B * W * 4 / (ms * 1e-3) / 1e9, 3)
    return out


def pmc_traffic(kernel):
    """HBM-side bytes per launch of `kernel` from the newest committed PMC
    summary (profiles/<round>_pmc.json, written by tools/pmc_summary.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def cpu_baseline(cfgname, seconds=12.0):
    """Oracle (numpy restatement of the reference step incl. its deque +
    random.sample replay) on the host, single BLAS thread, bounded sample."""
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
    n = 0
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        while True:
            b = O.sample_batch(buf, B)
            O.training_step(st, hp, b, erng.standard_normal((B, A_), dtype=np.float32),
                            erng.standard_normal((B, A_), dtype=np.float32))
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": round(n / el, 3), "unit": "gradient steps/s", "cores": 1, "kind": "port",
            "sample": f"{n} full training_step()s (deque+random.sample over {cap} rows, B={B}) in {el:.1f}s, "
                      "numpy fp32, 1 BLAS thread"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=device)

    from sac.replicas import replica_seed, timed_region

    seed = replica_seed(0, rank)
    eng, rb, c = build_engine(args.config, args.precision, seed, device)

    eng.train_graph(rb, args.warmup, args.chunk)
    eng.train_graph(rb, 0, args.chunk)  # capture the chunk graph now if warmup < chunk (runs no step)
    elapsed = timed_region(lambda: eng.train_graph(rb, args.steps, args.chunk), torch.cuda.synchronize, device)
    total_steps = args.steps * world
    eng.check()  # in-launch hand-offs all completed
    losses = eng.losses()
    if not all(np.isfinite(losses[:3])):
        raise SystemExit(f"non-finite losses after benchmark: {losses}")

    # per-phase device time (hipEvents on the launch stream), then roofline of the dominant kernel
    # Each interval also holds the cost of the event after it; the timed region
    # above ran the same launches from hipGraphs with no events.  The per-launch
    # event cost = (sum of the intervals of one step - the event-free step time)
    # / launches per step; interval - that cost = the kernel's own duration (the
    # figure rocprofv3 --kernel-trace reports: profiles/<round>_kernel_stats.csv).
    tp = eng.time_phases(rb, 100)
    phase_ms, empty_ms = tp[:4], tp[4]
    step_ms = elapsed / args.steps * 1e3
    n_launch = sum(1 for x in phase_ms if x > 0)
    ev_cost = max((sum(phase_ms) - step_ms) / n_launch, 0.0)
    kern_ms = [x - ev_cost if x > 0 else 0.0 for x in phase_ms]
    flops, f_total, _, _ = gemm_flops(c["obs"], c["act"], c["hidden"], c["batch"])
    if eng.fused:  # D inside the next A launch (and with layout 2, B inside the C launch)
        flops = [flops[0] + flops[3], flops[1], flops[2], 0]
        if eng.fused == 2:
            flops = [flops[0], 0, flops[2] + flops[1], 0]
    dom = int(np.argmax(phase_ms))
    from sac import _engine as E

    kname = E.load_library().sac_phase_kernel_name(dom).decode()
    traffic, traffic_src = pmc_traffic(kname) if args.config == "c2" and args.precision == "bf16" else (None, None)
    achieved = flops[dom] / (kern_ms[dom] * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]

    if rank == 0:
        sweep = {} if args.no_sweep else gather_sweep(rb, device)
        W = 2 * c["obs"] + c["act"] + 2
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
                                   "auto-alpha, device sampler",
                       "global_batch": c["batch"] * world, "parallelism": f"replicas{world}"},
            "replay_sample_GBps_in_step": round(sps / world * c["batch"] * W * 4 / 1e9, 4),
            "replay_sample_GBps_sweep": sweep,
            "phase_ms": [round(x, 5) for x in kern_ms],
            "phase_event_interval_ms": [round(x, 5) for x in phase_ms],
            "event_cost_ms": round(ev_cost, 5),
            "empty_kernel_event_interval_ms": round(empty_ms, 5),
            "step_gemm_flops_survey": f_total,
            "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "flops_per_launch": flops[dom],
                         "avg_launch_ms": round(kern_ms[dom], 5),
                         "timing": "hipEvents after every launch on the launch stream over 100 steps; "
                                   "avg_launch_ms = mean interval of this kernel's launches minus the per-launch "
                                   "event cost (event intervals of a step - event-free graph step time, per launch)"},
            "losses_last": [round(x, 6) for x in losses],
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
