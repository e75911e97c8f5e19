"""Probe: which rows of the bf16 row-tile kernels' log pi disagree with the
fp32 oracle (one step from the engine state), per shape; twice per engine
state (determinism)."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from oracle import sac_oracle as O  # noqa: E402
from test_gpu_parity import _oracle_state_from_engine  # noqa: E402

shapes = {"h128a6": dict(obs=24, act=6, hidden=[128, 128], batch=512, capacity=4096),
          "h128a4": dict(obs=24, act=4, hidden=[128, 128], batch=512, capacity=4096),
          "h64a6": dict(obs=24, act=6, hidden=[64, 64], batch=512, capacity=4096),
          "h192a6": dict(obs=24, act=6, hidden=[192, 192], batch=512, capacity=4096),
          "h128a2": dict(obs=24, act=2, hidden=[128, 128], batch=512, capacity=4096),
          "h128a6o8": dict(obs=8, act=6, hidden=[128, 128], batch=512, capacity=4096)}
lays = {"rows": {"layout": "rows"}, "roles": {"layout": "roles"}, "pairs": {"layout": "pairs"}}
for sname, c in shapes.items():
    for lname, lay in lays.items():
        bench.CONFIGS["_p"] = c
        try:
            eng, rb, cc = bench.build_engine("_p", "bf16", 3, torch.device("cuda", 0), layout=lay)
        except Exception as e:  # noqa: BLE001
            print(sname, lname, "build failed:", str(e)[:80])
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
        ref = O.training_step(st, hp, bt, et, ea)
        eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
                  eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, A))
        torch.cuda.synchronize()
        lp = eng.last_log_pi().cpu().numpy()
        y = eng.last_targets().cpu().numpy()
        r = np.abs(lp - ref["log_pi"]) / (np.abs(ref["log_pi"]) + 1)
        ry = np.abs(y - ref["y"]) / (np.abs(ref["y"]) + 1)
        bad = r > 0.05
        tiles = np.flatnonzero(bad.reshape(-1, 16).any(1))
        per_tile = bad.reshape(-1, 16).sum(1)
        print(f"{sname} {lname}: lp bad {bad.sum()}/{B} max {r.max():.2e}; y max {ry.max():.2e}; bad tiles {len(tiles)} "
              f"{tiles[:12].tolist()} rows-in-tile hist {np.bincount(np.flatnonzero(bad) % 16, minlength=16).tolist()}")
