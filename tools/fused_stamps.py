"""Where does the fused step (sac_persist.h) spend its time?  Runs C2 from the
-DSAC_STAMPS build (make -C soft-actor-critic_amd/csrc stamps) with the fused
step on and prints, per workgroup class of phase A (pi(s'), target critics,
critics, pi(s), spare), the median time of every STAMP point relative to the
launch's first stamp (s_memrealtime, 100 MHz; median over workgroups of the
class and over 10 steps).  A workgroup runs its phase A, B, C and D tasks in
that order; stamps 24 (A arrived), 25 (B counter seen), 26 (B arrived), 27 / 28
(C: pi(s) / critics' counter seen), 29 (C done), 30 (D counter seen), 31 (D
arrived) come from sac_persist.h, the others from the phase bodies."""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SAC_ENGINE_LIB", os.path.join(R, "soft-actor-critic_amd", "libsac_engine_stamps.so"))
os.environ.setdefault("SAC_PERSIST", "1")
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sac import _engine as E  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
dev = torch.device("cuda", 0)
bench.CONFIGS[cfg]["capacity"] = min(bench.CONFIGS[cfg]["capacity"], 100_000)
eng, rb, c = bench.build_engine(cfg, prec, 0, dev)
lib = E.load_library()
lib.sac_engine_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
lib.sac_engine_uses_fused_step.argtypes = [ctypes.c_void_p]
assert lib.sac_engine_debug_stamped() == 1, "not the stamps build"
G = lib.sac_engine_uses_fused_step(eng.handle)
assert G > 0, "fused step not in use"
nrt = (c["batch"] + 15) // 16
WP = 4 if prec == "fp32" else 2
classes = {"pi(s')": range(0, WP * nrt), "Qt": range(WP * nrt, (WP + 4) * nrt),
           "critic": range((WP + 4) * nrt, (WP + 8) * nrt), "pi(s)": range((WP + 8) * nrt, (WP + 10) * nrt),
           "spare": range((WP + 10) * nrt, G)}
buf = torch.zeros(G * 64, dtype=torch.int64, device=dev)
E.check(lib.sac_engine_debug_stamps(eng.handle, E.ptr(buf), eng._stream()))
eng.train(rb, 20)
torch.cuda.synchronize()
runs = []
for it in range(10):
    buf.zero_()
    eng.train(rb, 1)
    torch.cuda.synchronize()
    runs.append(buf.view(G, 64).cpu().numpy().copy())
names = {0: "A start", 8: "Qt2", 10: "Q1 fwd", 12: "Q2 fwd", 1: "A gather+eps", 2: "A L0", 3: "A L1", 4: "A L2", 6: "A published", 7: "Qt head",
         9: "Qt published", 16: "crit unit bwd", 15: "crit seed", 11: "Q1 GT stored", 13: "Q2 GT stored",
         24: "A arrived", 48: "B start", 25: "B saw AQ", 51: "B staged", 49: "B dW", 50: "B adam", 26: "B arrived",
         32: "C start", 27: "C saw PS", 28: "C saw BQ", 33: "C inputs", 36: "C Q1 fwd", 37: "C Q2 fwd",
         38: "C Q1 da", 34: "C pi inputs", 39: "C pi combined", 35: "C pi bwd", 29: "C done",
         52: "D start", 30: "D saw CP", 55: "D staged", 53: "D dW", 54: "D adam", 31: "D arrived", 60: "END"}
print(f"fused step {cfg} {prec}: G = {G} workgroups, medians in us from the launch's first stamp")
spans = []
for r in runs:
    v = r[r > 0]
    spans.append((v.max() - v.min()) / 100.0)
print(f"launch span (first stamp -> last END): median {np.median(spans):.2f} us")
for cname, rng in classes.items():
    if len(rng) == 0:
        continue
    line = []
    for i in sorted(names, key=lambda i: np.median([np.median(r[list(rng), i][r[list(rng), i] > 0] - r[r > 0].min())
                                                    if (r[list(rng), i] > 0).any() else 1e18 for r in runs])):
        vals = []
        for r in runs:
            t0 = r[r > 0].min()
            col = r[list(rng), i]
            col = col[col > 0]
            if col.size:
                vals.append(np.median(col - t0) / 100.0)
        if vals:
            mx = np.median([(r[list(rng), i][r[list(rng), i] > 0].max() - r[r > 0].min()) / 100.0
                            for r in runs if (r[list(rng), i] > 0).any()])
            line.append(f"{names[i]} {np.median(vals):.2f}/{mx:.2f}")
    print(f"[{cname:7s}] " + " | ".join(line))
print("(median / max over the class's workgroups, each the median over steps)")
last = [np.unravel_index(np.argmax(r), r.shape) for r in runs]
print("last stamp of the launch (workgroup, stamp id) per step:", [(int(w), int(i)) for w, i in last])
