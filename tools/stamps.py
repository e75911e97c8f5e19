"""Where does a phase kernel spend its time?  Runs the C2 engine from the
-DSAC_STAMPS build (make -C soft-actor-critic_amd/csrc stamps) and prints, per
phase and per workgroup role, the time between STAMP(i) points in microseconds
(s_memrealtime, 100 MHz, one clock for every XCD; median over row tiles and over
10 steps), then a launch-wide timeline relative to the launch's first stamp."""
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
# optional "layout=NAME" argument: a kernel layout override (e.g. layout=pairs)
lay = [a.split("=", 1)[1] for a in sys.argv[3:] if a.startswith("layout=")]
eng, rb, c = bench.build_engine(cfg, prec, 0, dev, layout={"layout": lay[0]} if lay else None)
lib = E.load_library()
lib.sac_engine_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
assert lib.sac_engine_debug_stamped() == 1, "not the stamps build"
nblk = 2048  # rows for every block index any phase grid can have (B/D tile grids included)
nrt = (c["batch"] + 15) // 16


def _tiles(dims):
    return sum(((dims[i + 1] + 31) // 32) * ((dims[i] + 31) // 32) for i in range(len(dims) - 1))


O_, A_, H_ = c["obs"], c["act"], c["hidden"]
n_b = 2 * _tiles([O_ + A_] + H_ + [1])
n_d = _tiles([O_] + H_ + [2 * A_])
OFF = {"A": 0, "C": 0}  # role blocks are the launches' first blocks
lib.sac_engine_uses_split.argtypes = [ctypes.c_void_p]
SPLIT = bool(lib.sac_engine_uses_split(eng.handle))
lib.sac_engine_uses_pairs.argtypes = [ctypes.c_void_p]
PAIRS = bool(lib.sac_engine_uses_pairs(eng.handle))
GROUP = 2 * nrt if SPLIT else nrt  # blocks per role group (hidden split: two halves per row tile in A)
GROUP_C = 4 * nrt if SPLIT else nrt  # phase C: the critic roles' parts per row tile (split_wcq; pi: the rest)
buf = torch.zeros(nblk * 64, dtype=torch.int64, device=dev)
E.check(lib.sac_engine_debug_stamps(eng.handle, E.ptr(buf), eng._stream()))
eng.train(rb, 20)
torch.cuda.synchronize()
# mode "rerun": after each step, phase A launched again right behind itself
# (instruction cache warm from the first A) and only that second A is stamped.
# Timing experiment: the extra A advances the training state out of sequence.
# mode "rerunC": the same with phase C (weights read by the first C are warm for the second)
rerun = len(sys.argv) > 3 and sys.argv[3] in ("rerun", "rerunC")
rerun_kind = 2 if rerun and sys.argv[3] == "rerunC" else 0
if rerun:
    lib.sac_engine_debug_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    desc = rb.desc
runs = []
for it in range(10):
    buf.zero_()
    eng.train(rb, 1)
    if rerun:
        E.check(lib.sac_engine_debug_launch(eng.handle, ctypes.byref(desc), rerun_kind, eng._stream()))
        torch.cuda.synchronize()
        buf.zero_()
        E.check(lib.sac_engine_debug_launch(eng.handle, ctypes.byref(desc), rerun_kind, eng._stream()))
    torch.cuda.synchronize()
    runs.append(buf.view(nblk, 64).cpu().numpy().copy())
names = {58: "D done", 59: "D waited",
         0: "start", 1: "gather+eps", 56: "pi X built", 57: "pi L0 issued", 2: "pi L0", 3: "pi L1", 4: "pi L2",
         5: "pi L3", 6: "head+publish", 7: "Qt1", 8: "Qt2", 9: "Qt published", 10: "Q1 fwd", 12: "Q2 fwd",
         16: "unit bwd", 14: "y inputs in", 15: "seed", 11: "Q1 GT stored", 13: "Q2 GT stored",
         32: "start", 36: "Q1 fwd", 37: "Q2 fwd", 38: "Q1 bwd->da", 39: "Q2 bwd->da / combined", 35: "pi bwd",
         48: "start", 49: "dW", 50: "adam", 52: "start", 53: "dW", 54: "adam", 51: "staged", 55: "staged"}
names.update({33: "B waited", 20: "HC8 layer entry", 21: "HC8 MFMA done (wave 0)", 22: "HC8 epilogue done",
              23: "HC8 layer end"})
names.update({60: "END", 61: "END", 62: "END", 63: "END"})
if SPLIT:  # sac_split.h stamps
    names.update({2: "L0", 3: "L1 half", 4: "L2 partial", 6: "partials published", 7: "pi head (s')",
                  9: "Qt partial published", 33: "inputs", 34: "pi inputs", 36: "Q1 fwd", 37: "Q2 fwd",
                  38: "Q1 da partial", 39: "pi: critics combined", 35: "pi bwd + GT"})
    names.update({20: "kernel entry", 21: "step loaded", 22: "record in registers"})
if PAIRS:  # sac_pairs.h stamps
    names.update({6: "pi(s') head", 7: "Qt1", 8: "Qt2 + y", 9: "pi(s) + stashes", 14: "seeds (critics polled)",
                  10: "Q1 fwd", 11: "Q1 bwd + GT", 12: "Q2 fwd", 13: "Q2 bwd + GT", 33: "inputs",
                  36: "Q1 fwd", 37: "Q2 fwd", 38: "Q1 da", 39: "Q2 da published / combined", 35: "pi bwd + GT"})
    GROUP = GROUP_C = (nrt + 1) // 2  # pair tiles per group
WPI = (4 if prec == "fp32" else 2) if SPLIT else 1  # phase A: pi(s') parts (split_wpi)


# phase A's split kernel places each weight part's workgroups on one or two XCDs
# (EngineDev::role_xcd, default on): hardware block -> the body's block id
ROLE_XCD = SPLIT and (10 + WPI) * nrt % 8 == 0


def _role_xcd_bid(b):
    n0, n2, G = WPI * nrt, 2 * nrt, (10 + WPI) * nrt
    u = (b % 8) * (G // 8) + b // 8
    v = u - n0
    return np.where(u < n0, (u % nrt) * WPI + u // nrt, n0 + (v // n2) * n2 + (v % n2 % nrt) * 2 + v % n2 // nrt)


def role_of(ph, b, G):
    """Role index of phase-relative block ids b (phase A: pi(s') has WPI parts per row tile)."""
    if ph == "A" and SPLIT:
        n0 = WPI * nrt
        if ROLE_XCD:
            b = _role_xcd_bid(np.asarray(b))
        return np.where(b < n0, 0, 1 + (b - n0) // G)
    return b // G


PH = {"A": list(range(0, 17)) + [20, 21, 22, 23, 56, 57, 59, 60],  # 20-23: free for DSTAMP probes
      "C": list(range(32, 40)) + [61], "B": [48, 51, 49, 50, 62], "D": [52, 55, 53, 54, 63]}
ROLES = {"A": ["pi(s')", "Qt1", "Qt2", "Q1", "Q2", "pi(s)"], "C": ["Q1", "Q2", "pi"]}  # block-group order
if PAIRS:
    ROLES = {"A": ["critics", "target + pi(s)"], "C": ["Q2", "Q1 + pi"]}
# shader clock during phase A: s_memtime ticks (slots 40/41) per realtime tick (slots 0/60)
clk = []
for r in runs:
    m = (r[:, 40] > 0) & (r[:, 41] > 0) & (r[:, 60] > r[:, 0])
    clk += list((r[m, 41] - r[m, 40]) / ((r[m, 60] - r[m, 0]) / 100.0))
if clk:
    print(f"phase A shader clock: {np.median(clk):.0f} MHz (median over blocks)")
for ph, ids in PH.items():
    base = ids[0]
    rows = np.concatenate([r[r[:, base] > 0] for r in runs])
    blk = np.concatenate([np.nonzero(r[:, base] > 0)[0] for r in runs])
    if rows.size == 0:
        continue
    groups = {"all": np.ones(len(blk), bool)}
    if ph in ROLES and (eng.roles or PAIRS):
        rb_ = blk - OFF[ph]
        G = GROUP_C if ph == "C" else GROUP
        ridx = role_of(ph, rb_, G)
        groups = {nm: (rb_ >= 0) & (ridx == k) for k, nm in enumerate(ROLES[ph])}
        if OFF[ph]:
            groups["upd"] = rb_ < 0
    print(f"=== phase {ph}")
    endc = {"A": 60, "C": 61, "B": 62, "D": 63}[ph]
    spans = []
    for r in runs:
        live = r[:, base] > 0
        if live.any() and (r[live, endc] > 0).any():
            spans.append(r[live, endc].max() - r[live, base].min())
    if spans:
        print(f"  launch span (first block start -> last block end, stores drained): {np.median(spans) / 100:.2f} us")
        st_, en_ = [], []
        for r in runs:
            live = r[:, base] > 0
            if live.any() and (r[live, endc] > 0).all():
                t0 = r[live, base].min()
                st_.append(r[live, base] - t0)
                en_.append(r[live, endc] - t0)
        if st_:
            st_, en_ = np.concatenate(st_) / 100, np.concatenate(en_) / 100
            q = lambda x: " ".join(f"{v:.2f}" for v in np.percentile(x, [0, 25, 50, 75, 90, 100]))  # noqa: E731
            print(f"  block start (us, p0 p25 p50 p75 p90 p100): {q(st_)}")
            print(f"  block end   (us, p0 p25 p50 p75 p90 p100): {q(en_)}")
            r = runs[-1]
            live = np.nonzero(r[:, base] > 0)[0]
            t0 = r[live, base].min()
            late = sorted(live, key=lambda b: -r[b, endc])[:12]
            print("  latest blocks (id: start/end us): " + ", ".join(
                f"{b}: {(r[b, base] - t0) / 100:.2f}/{(r[b, endc] - t0) / 100:.2f}" for b in late))
            if ph in ("B", "D"):
                for b in list(late[:3]) + [int(np.median(live))]:
                    print(f"    block {b}: " + " | ".join(f"{names.get(i, i)} {(r[b, i] - t0) / 100:.2f}"
                                                      for i in ids if r[b, i] > 0))
    for g, m in groups.items():
        if not m.any():
            continue
        sel = rows[m]
        seq = [(i, np.median(sel[sel[:, i] > 0, i] - sel[sel[:, i] > 0, base])) for i in ids
               if i != base and (sel[:, i] > 0).any()]
        seq.sort(key=lambda x: x[1])
        line, prev = [], 0.0
        for i, t in seq:
            line.append(f"{names.get(i, i)} +{(t - prev) / 100:.2f}")
            prev = t
        print(f"  [{g:6s}] " + " | ".join(line) + f"   (total {prev / 100:.2f} us)")
        # absolute: each stamp relative to the launch's earliest stamp of this phase
        ab = []
        for i in ids:
            vals = []
            for r in runs:
                live = r[:, base] > 0
                t0 = r[live, base].min()
                bm = np.zeros(len(r), bool)
                bm[np.nonzero(live)[0]] = True
                sel_r = r[bm]
                blk_r = np.nonzero(bm)[0]
                gm = np.ones(len(blk_r), bool)
                if ph in ROLES and eng.roles:
                    rb2 = blk_r - OFF[ph]
                    k = list(groups).index(g) if g in ROLES.get(ph, []) else -1
                    G = GROUP_C if ph == "C" else GROUP
                    gm = (rb2 >= 0) & (role_of(ph, rb2, G) == k) if k >= 0 else (rb2 < 0)
                v = sel_r[gm, i]
                v = v[v > 0]
                if v.size:
                    vals.append(np.median(v) - t0)
            if vals:
                ab.append((np.median(vals), names.get(i, i)))
        ab.sort()
        print("           @ " + " | ".join(f"{n} {t / 100:.2f}" for t, n in ab))
