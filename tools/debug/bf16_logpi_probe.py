"""Probe: bf16 log pi of one step from the engine's state vs the fp32 oracle,
per layout, at a given shape; prints the worst rows."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from oracle import sac_oracle as O  # noqa: E402
from test_gpu_parity import _oracle_state_from_engine  # noqa: E402

shapes = {"s17": dict(obs=17, act=6, hidden=[128, 128], batch=2000, capacity=4096),
          "s24": dict(obs=24, act=4, hidden=[256, 256], batch=2000, capacity=4096),
          "s17h256": dict(obs=17, act=6, hidden=[256, 256], batch=2000, capacity=4096),
          "s24a6": dict(obs=24, act=6, hidden=[128, 128], batch=2000, capacity=4096)}
for sname, c in shapes.items():
    for lay in ({"layout": "rows"}, {"layout": "pairs"}, {"stage_path": 1}):
        for prec in ("bf16", "fp32"):
            bench.CONFIGS["_p"] = c
            try:
                eng, rb, cc = bench.build_engine("_p", prec, 3, torch.device("cuda", 0), layout=lay)
            except Exception as e:  # noqa: BLE001
                print(sname, lay, prec, "build failed:", e)
                continue
            finally:
                del bench.CONFIGS["_p"]
            B, A = cc["batch"], cc["act"]
            hp = O.SacHyper(alpha=0.1, auto_entropy_tuning=True)
            rows = {k: getattr(rb, k).cpu().numpy() for k in ("obs", "act", "rew", "next_obs", "done")}
            g = np.random.default_rng(13)
            st = _oracle_state_from_engine(eng, A)
            idx = g.choice(len(rb), size=B, replace=False).astype(np.int32)
            et = g.standard_normal((B, A)).astype(np.float32)
            ea = g.standard_normal((B, A)).astype(np.float32)
            bt = O.Batch(rows["obs"][idx], rows["act"][idx], rows["rew"][idx], rows["next_obs"][idx], rows["done"][idx])
            _, _, ctx = O.policy_sample(st.pi, bt.s, ea, hp.policy)
            ref = O.training_step(st, hp, bt, et, ea)
            eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
                      eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, A))
            torch.cuda.synchronize()
            lp = eng.last_log_pi().cpu().numpy()
            r = np.abs(lp - ref["log_pi"]) / (np.abs(ref["log_pi"]) + 1)
            w = np.argsort(-r)[:5]
            print(sname, lay, prec, "pairs" if eng.pairs else "", "wide" if eng.wide else "",
                  f"lp rel p50 {np.median(r):.2e} p99 {np.quantile(r, .99):.2e} max {r.max():.2e} n>0.1 {(r > 0.1).sum()}")
            for b in w[:3]:
                print("   row", b, "eng", lp[b], "ora", ref["log_pi"][b], "ls", ctx["log_std"][b], "mu", ctx["mu"][b],
                      "eps", ea[b])
