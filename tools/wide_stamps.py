"""Where does a GEMM stage of the large-batch path (csrc/sac_wide.h) spend its
time?  Runs the engine from the -DSAC_STAMPS build with SAC_WIDE_STAMP_STAGE=k
for each requested stage k and prints, over the stage's workgroups: the spread
of their start times, the median time between stamp points (prologue, first K
block in LDS, each K block, epilogue tile, stores drained) and the launch span.
    python tools/wide_stamps.py [config] [precision] [stage ...]"""
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

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
stages = [int(x) for x in sys.argv[3:]] or [1, 2, 4, 5, 6, 8, 9, 10, 11]
dev = torch.device("cuda", 0)
bench.CONFIGS[cfg]["capacity"] = min(bench.CONFIGS[cfg]["capacity"], 100_000)
NAMES = {0: "entry", 1: "prologue", 2: "K block 0 in LDS", 11: "K loop done", 12: "epilogue tile", 13: "stores drained"}
NAMES.update({3 + k: f"K block {k + 1}" for k in range(8)})
for st in stages:
    os.environ["SAC_WIDE_STAMP_STAGE"] = str(st)
    eng, rb, c = bench.build_engine(cfg, prec, 0, dev)
    lib = E.load_library()
    assert lib.sac_engine_debug_stamped() == 1, "not the stamps build"
    lib.sac_engine_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    nblk = 4096
    buf = torch.zeros(nblk * 64, dtype=torch.int64, device=dev)
    E.check(lib.sac_engine_debug_stamps(eng.handle, E.ptr(buf), eng._stream()))
    eng.train(rb, 5)
    spans, rows = [], []
    for it in range(5):
        buf.zero_()
        eng.train(rb, 1)
        torch.cuda.synchronize()
        s = buf.view(nblk, 64).cpu().numpy().copy()
        live = s[:, 0] > 0
        s = s[live]
        t0 = s[:, 0].min()
        spans.append((s[:, 13].max() - t0) / 100.0)
        rows.append((s - t0) / 100.0)
    a = np.concatenate(rows)
    starts = a[:, 0]
    print(f"=== stage {st} ({cfg} {prec}): {a.shape[0] // 5} workgroups, span {np.median(spans):.2f} us")
    print("  block start (us, p0 p50 p90 p100): " + " ".join(f"{np.percentile(starts, q):.2f}" for q in (0, 50, 90, 100)))
    pts = [i for i in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13) if np.all(a[:, i] > -1e-9) and np.any(a[:, i] > 0)]
    prev = 0
    out = []
    for i in pts[1:]:
        d = np.median(a[:, i] - a[:, prev])
        out.append(f"{NAMES.get(i, i)} +{d:.2f}")
        prev = i
    print("  " + " | ".join(out))
    print("  block end (us, p50 p90 p100): " + " ".join(f"{np.percentile(a[:, 13], q):.2f}" for q in (50, 90, 100)))
    eng.close()
    del eng, rb
    torch.cuda.empty_cache()
