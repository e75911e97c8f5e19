"""How does the one-block-per-row-tile kernel (C3 shapes) scale with the number
of row tiles?  Per-phase event intervals (ms) at batch 4096 / 2048 / 1024 / 512:
a launch whose time stays flat as blocks halve is bound per CU; one whose time
falls with the block count is bound by a shared resource (Infinity Cache / HBM)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
for batch in (4096, 2048, 1024, 512):
    bench.CONFIGS["c3"]["batch"] = batch
    bench.CONFIGS["c3"]["capacity"] = 100_000
    eng, rb, c = bench.build_engine("c3", prec, 0, dev)
    eng.train_graph(rb, 20, 10)
    tp = eng.time_phases(rb, 50)
    print(prec, batch, "roles" if eng.roles else "rowtile", [round(x * 1e3, 2) for x in tp[:5]], flush=True)
    del eng, rb
