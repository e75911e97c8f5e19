"""K independent-seed SAC learners on ONE MI355X, one HIP stream each (C2).

One learner's step is a latency chain that occupies at most 96 of the 256 CUs
(DESIGN.md §5), so independent learners (SURVEY §8e replicas, packed per GPU
instead of one per GPU) can share a device.  Every learner runs full C2 steps
(own weights, own replay, own Philox stream); nothing is skipped.  Prints
aggregate gradient steps/s for each K as one JSON line.  This is NOT
bench.py's headline value (one learner's steps/s).

    python tools/multi_learner_bench.py [--ks 1,2,4,8] [--steps 1000]
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--capacity", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bench.CONFIGS["c2"]["capacity"] = args.capacity
    ks = [int(k) for k in args.ks.split(",")]
    learners = []
    for i in range(max(ks)):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            eng, rb, _ = bench.build_engine("c2", "bf16", i, dev)
            eng.train_graph(rb, 2 * args.chunk, args.chunk)  # warm-up + graph capture
        learners.append((s, eng, rb))
        print(f"learner {i} ready", flush=True)
    torch.cuda.synchronize()
    out = {"config": "c2 bf16, own replay per learner", "capacity": args.capacity,
           "steps_per_learner": args.steps, "results": {}}
    for k in ks:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, eng, rb in learners[:k]:
            with torch.cuda.stream(s):
                eng.train_graph(rb, args.steps, args.chunk)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        for _, eng, _ in learners[:k]:
            eng.check()
        out["results"][str(k)] = {"aggregate_steps_per_s": round(k * args.steps / el, 1),
                                  "per_learner_steps_per_s": round(args.steps / el, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
