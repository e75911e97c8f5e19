"""The driver's short form (--steps 20 --warmup 5) timed several ways on one
engine: one 20-step graph replay (bench.py's timed region), the same 20 steps
as eager launches, and the replay with the host's second synchronize removed
from the timed region.  Median over repeats, steps/s."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
dev = torch.device("cuda", 0)
eng, rb, c = bench.build_engine("c2", prec, 0, dev)
eng.train_graph(rb, 0, 20)
bench.prewarm(rb, dev, 0.3)
eng.train_graph(rb, 5, 20)
sync = torch.cuda.synchronize
res = {"graph_2sync": [], "graph_1sync": [], "eager": []}
for rep in range(12):
    for form in res:
        sync()
        sync()
        t0 = time.perf_counter()
        if form == "eager":
            eng.train(rb, 20)
        else:
            eng.train_graph(rb, 20, 20)
        sync()
        if form == "graph_2sync":
            sync()
        el = time.perf_counter() - t0
        res[form].append(20 / el)
print({k: round(float(np.median(v)), 1) for k, v in res.items()}, {k: round(float(np.max(v)), 1) for k, v in res.items()})
