"""Where does a phase kernel spend its time?  Runs the C2 engine from the
-DSAC_STAMPS build (make -C soft-actor-critic_amd/csrc stamps) and prints the
s_memtime deltas between the STAMP(i) points, median over row-tile blocks."""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SAC_ENGINE_LIB", os.path.join(R, "soft-actor-critic_amd", "libsac_engine_stamps.so"))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sac import _engine as E  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
dev = torch.device("cuda", 0)
bench.CONFIGS[cfg]["capacity"] = min(bench.CONFIGS[cfg]["capacity"], 100_000)
eng, rb, c = bench.build_engine(cfg, prec, 0, dev)
lib = E.load_library()
lib.sac_engine_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
assert lib.sac_engine_debug_stamped() == 1, "not the stamps build"
nblk = 2048  # rows for every block index any phase grid can have (B/D tile grids included)
buf = torch.zeros(nblk * 64, dtype=torch.int64, device=dev)
E.check(lib.sac_engine_debug_stamps(eng.handle, E.ptr(buf), eng._stream()))
eng.train(rb, 20)
torch.cuda.synchronize()
rows = []
for it in range(10):
    buf.zero_()
    eng.train(rb, 1)
    torch.cuda.synchronize()
    rows.append(buf.view(nblk, 64).cpu().numpy())
st = np.median(np.stack(rows), axis=0)  # [blk][64]
names = {0: "A start", 1: "gather+eps", 2: "pi L0", 3: "pi L1", 4: "pi L2", 5: "pi L3", 6: "head",
         7: "Qt1", 8: "Qt2", 9: "Qt published", 10: "Q1 fwd", 11: "Q1 bwd", 12: "Q2 fwd", 13: "Q2 bwd",
         14: "y inputs in", 15: "seed", 16: "unit bwd",
         32: "C start", 36: "Q1 fwd", 37: "Q2 fwd", 38: "Q1 bwd->da", 39: "Q2 bwd->da", 35: "pi bwd"}
names.update({48: "B start", 49: "B dW done", 50: "B adam issued", 52: "D start", 53: "D dW done",
              54: "D adam issued"})
for base, last in ((0, 16), (32, 39), (48, 50), (52, 54)):
    live = st[:, base] > 0  # blocks that ran this phase
    idx = [i for i in range(base, last + 1) if i in names and (st[live, i] > 0).any()]
    idx.sort(key=lambda i: np.median(st[live & (st[:, i] > 0), i] - st[live & (st[:, i] > 0), base]))
    prev = None
    print(f"--- phase {dict([(0, 'A'), (32, 'C'), (48, 'B'), (52, 'D')])[base]} (cycles, median over blocks)")
    for i in idx:
        m = live & (st[:, i] > 0)
        t = np.median(st[m, i] - st[m, base])
        if prev is not None:
            print(f"  {names[i]:12s} +{t - prev:9.0f}   (cum {t:9.0f})")
        prev = t

# whole-grid view: first start -> last stamp of each phase (dispatch skew + slowest block)
for base, last, nm in ((0, 16, "A"), (32, 39, "C"), (48, 50, "B"), (52, 54, "D")):
    live = st[:, base] > 0
    if not live.any():
        continue
    t0 = st[live, base].min()
    ends = st[live, base:last + 1].max(axis=1)
    print(f"--- phase {nm}: blocks {live.sum()}, start skew {st[live, base].max() - t0:.0f}, "
          f"span first-start -> last-stamp {ends.max() - t0:.0f} cycles")
