"""Debug: ONE-step parity from the engine's own full state (parameters, Adam
moments and step counts, alpha state): the oracle runs step k+1 from the state
the engine reached after step k, and the engine's post-step parameters are
compared with it.  Separates the kernels' per-step arithmetic from trajectory
drift.  python tools/debug/local_step.py OBS ACT H1,H2 B"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "soft-actor-critic_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from oracle import sac_oracle as O  # noqa: E402

obs, act = int(sys.argv[1]), int(sys.argv[2])
hidden = [int(x) for x in sys.argv[3].split(",")]
B = int(sys.argv[4])
bench.CONFIGS["_dbg"] = dict(obs=obs, act=act, hidden=hidden, batch=B, capacity=max(2048, 2 * B))
eng, rb, cc = bench.build_engine("_dbg", "fp32", 3, torch.device("cuda", 0))
print(sys.argv[1:], "roles", eng.roles, flush=True)
hp = O.SacHyper(alpha=0.1, auto_entropy_tuning=True)
rows = {k: getattr(rb, k).cpu().numpy() for k in ("obs", "act", "rew", "next_obs", "done")}
np_ = lambda t: t.detach().cpu().numpy().copy()  # noqa: E731


def engine_state():
    mlp = {k: O.MLP.from_state_dict({kk: np_(v) for kk, v in eng.nets[k].state_dict().items()}, "relu")
           for k in ("pi", "q1", "q2", "q1t", "q2t")}
    steps = eng.opt_steps.cpu().numpy()
    opt = {}
    for i, k in enumerate(("pi", "q1", "q2")):
        m, v = eng.adam_views(k)
        opt[k] = O.AdamState([np_(x) for x in m], [np_(x) for x in v], float(steps[i]))
    al = eng.alpha_state.cpu().numpy()
    st = O.SacState(mlp["pi"], mlp["q1"], mlp["q2"], mlp["q1t"], mlp["q2t"], opt["pi"], opt["q1"], opt["q2"], act,
                    log_alpha=float(al[0]), alpha=float(al[1]), opt_alpha_m=float(al[2]), opt_alpha_v=float(al[3]),
                    opt_alpha_step=float(steps[3]))
    return st


def f64_pi_update(pre_pi, mo, idx, ea):
    """float64 torch: the actor step's update of pi's layer-0 weight from the
    engine's pre-step pi and Adam state, through the engine's post-step critics
    (the reference updates the critics first)."""
    import torch.nn.functional as F
    d = torch.float64
    W = [torch.tensor(pre_pi[f"net.{2 * i}.weight"], dtype=d, requires_grad=True) for i in range(len(hidden) + 1)]
    b = [torch.tensor(pre_pi[f"net.{2 * i}.bias"], dtype=d, requires_grad=True) for i in range(len(hidden) + 1)]
    s = torch.tensor(rows["obs"][idx], dtype=d)
    h = s
    for i in range(len(W)):
        h = h @ W[i].T + b[i]
        if i < len(W) - 1:
            h = torch.relu(h)
    raw = h[:, act:].detach()
    print(f"      f64 head: log_std raw range [{raw.min():.2f}, {raw.max():.2f}] clamped {(raw > 2).sum().item()}"
          f" |mu|max {h[:, :act].abs().max().item():.2f}", flush=True)
    mu, ls = h[:, :act], torch.clamp(h[:, act:], -20.0, 2.0)
    sd = ls.exp()
    e = torch.tensor(ea, dtype=d)
    z = mu + e * sd
    a = torch.tanh(z)
    lp = (-((z - mu) ** 2) / (2 * sd * sd) - ls - 0.5 * np.log(2 * np.pi)).sum(1)
    lp = lp - (2 * (np.log(2) - z - F.softplus(-2 * z))).sum(1)
    def q(key):
        sd_ = {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets[key].state_dict().items()}
        x = torch.cat([s, a], 1)
        n = len(hidden) + 1
        for i in range(n):
            x = x @ sd_[f"net.{2 * i}.weight"].T + sd_[f"net.{2 * i}.bias"]
            if i < n - 1:
                x = torch.relu(x)
        return x[:, 0]
    alpha = float(alpha_pre)
    qa, qb = q("q1"), q("q2")
    gap = (qa - qb).abs().detach()
    print(f"      f64 min-Q: smallest |q1 - q2| {gap.min().item():.3e} (row {int(gap.argmin())}),"
          f" rows under 1e-5: {(gap < 1e-5).sum().item()}", flush=True)
    loss = (alpha * lp - torch.minimum(qa, qb)).mean()
    loss.backward()
    g = W[0].grad.numpy()
    m0, v0 = mo[0][0].astype(np.float64), mo[1][0].astype(np.float64)
    t = float(steps_pre[0]) + 1.0
    m = 0.9 * m0 + 0.1 * g
    v = 0.999 * v0 + 0.001 * g * g
    return -(3e-4 / (1 - 0.9 ** t)) * m / (np.sqrt(v) / np.sqrt(1 - 0.999 ** t) + 1e-8)


g = np.random.default_rng(int(os.environ.get("DBG_SEED", "11")))
for k in range(1, 5):
    idx = g.choice(len(rb), size=B, replace=False).astype(np.int32)
    et = g.standard_normal((B, act)).astype(np.float32)
    ea = g.standard_normal((B, act)).astype(np.float32)
    st = engine_state()
    pre_pi = {kk: np_(v) for kk, v in eng.nets["pi"].state_dict().items()}
    alpha_pre = eng.alpha_state.cpu().numpy()[1]
    steps_pre = eng.opt_steps.cpu().numpy()
    mo = ([x.copy() for x in st.opt_pi.m], [x.copy() for x in st.opt_pi.v])
    ref = O.training_step(st, hp, O.Batch(rows["obs"][idx], rows["act"][idx], rows["rew"][idx],
                                          rows["next_obs"][idx], rows["done"][idx]), et, ea)
    eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
              eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, act))
    torch.cuda.synchronize()
    print(f"step {k} losses", np.round(np.array(eng.losses()), 6), np.round(np.array(ref["losses"]), 6))
    for n, net in (("pi", st.pi), ("q1", st.q1), ("q2", st.q2), ("q1t", st.q1t), ("q2t", st.q2t)):
        mine = {kk: v.detach().cpu().numpy() for kk, v in eng.nets[n].state_dict().items()}
        parts = []
        for pk, want in net.state_dict().items():
            d = np.abs(mine[pk] - want)
            parts.append(f"{pk}:{np.mean(d <= 1e-6):.3f}/{d.max():.1e}")
        print(f"   {n}: " + " ".join(parts), flush=True)
        if n == "pi":
            w_e, w_o = mine["net.0.weight"], net.state_dict()["net.0.weight"]
            upd64 = f64_pi_update(pre_pi, mo, idx, ea)
            w0 = pre_pi["net.0.weight"].astype(np.float64)
            de, do = w_e - w0, w_o - w0
            bad = np.abs(w_e - w_o) > 1e-6
            print(f"      pi L0 off {bad.sum()}: |engine - f64| max {np.abs(de - upd64).max():.2e} mean {np.abs(de - upd64).mean():.2e};"
                  f" |oracle - f64| max {np.abs(do - upd64).max():.2e} mean {np.abs(do - upd64).mean():.2e}", flush=True)
