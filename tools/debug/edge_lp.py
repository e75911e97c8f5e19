"""Debug: per-step y / log pi deviation of the engine from the oracle at an edge
shape (tests/test_gpu_parity.py EDGE_SHAPES), fp32."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "soft-actor-critic_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from oracle import sac_oracle as O  # noqa: E402

obs, act = int(sys.argv[1]), int(sys.argv[2])
env = sys.argv[3] if len(sys.argv) > 3 else ""
if env:
    k_, v_ = env.split("=")
    os.environ[k_] = v_
bench.CONFIGS["_dbg"] = dict(obs=obs, act=act, hidden=[256, 256], batch=64, capacity=1024)
eng, rb, cc = bench.build_engine("_dbg", "fp32", 3, torch.device("cuda", 0))
print("roles", eng.roles, "split", getattr(eng, "split", None))
B, A = cc["batch"], cc["act"]
sds = {k: {kk: v.detach().cpu().numpy().copy() for kk, v in m.state_dict().items()} for k, m in eng.nets.items()}
hp = O.SacHyper(alpha=0.1, auto_entropy_tuning=True)
st = O.SacState.fresh(O.MLP.from_state_dict(sds["pi"], "relu"), O.MLP.from_state_dict(sds["q1"], "relu"),
                      O.MLP.from_state_dict(sds["q2"], "relu"), hp, A)
rows = {k: getattr(rb, k).cpu().numpy() for k in ("obs", "act", "rew", "next_obs", "done")}
g = np.random.default_rng(11)
for k in range(1, 4):
    idx = g.choice(len(rb), size=B, replace=False).astype(np.int32)
    et = g.standard_normal((B, A)).astype(np.float32)
    ea = g.standard_normal((B, A)).astype(np.float32)
    ref = O.training_step(st, hp, O.Batch(rows["obs"][idx], rows["act"][idx], rows["rew"][idx],
                                          rows["next_obs"][idx], rows["done"][idx]), et, ea)
    eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
              eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, A))
    torch.cuda.synchronize()
    y = eng.last_targets().cpu().numpy()
    lp = eng.last_log_pi().cpu().numpy()
    dy = np.abs(y - ref["y"])
    dl = np.abs(lp - ref["log_pi"])
    bad = np.argsort(-dl)[:5]
    print(f"step {k}: y max {dy.max():.3e}  lp max {dl.max():.3e} mean {dl.mean():.3e}  worst rows {bad.tolist()}"
          f" lp {lp[bad].round(4).tolist()} want {ref['log_pi'][bad].round(4).tolist()}")
    print("   losses", np.array(eng.losses()), np.array(ref["losses"]))
