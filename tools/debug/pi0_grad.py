"""Debug: pi's layer-0 weight gradient of one step, engine vs float64.
The engine's gradient is recovered from its post-step Adam moment
(exp_avg_new = b1 exp_avg + (1 - b1) g), float64 torch recomputes the actor
loss gradient from the engine's pre-step pi, its post-step critics and the
step's batch and eps (as tools/debug/local_step.py).  Prints the relative
error per 32 x 32 update tile and the worst rows / columns.
    python tools/debug/pi0_grad.py OBS ACT H1,H2 B [steps]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "soft-actor-critic_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402

obs, act = int(sys.argv[1]), int(sys.argv[2])
hidden = [int(x) for x in sys.argv[3].split(",")]
B = int(sys.argv[4])
nsteps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
bench.CONFIGS["_dbg"] = dict(obs=obs, act=act, hidden=hidden, batch=B, capacity=max(2048, 2 * B))
eng, rb, cc = bench.build_engine("_dbg", "fp32", 3, torch.device("cuda", 0))
print(sys.argv[1:], "roles", eng.roles, "wide", eng.wide, flush=True)
rows = {k: getattr(rb, k).cpu().numpy() for k in ("obs", "act", "rew", "next_obs", "done")}
np_ = lambda t: t.detach().cpu().numpy().copy()  # noqa: E731
d = torch.float64


def mlp64(sd, x, n):
    for i in range(n):
        x = x @ sd[f"net.{2 * i}.weight"].T + sd[f"net.{2 * i}.bias"]
        if i < n - 1:
            x = torch.relu(x)
    return x


g = np.random.default_rng(int(os.environ.get("DBG_SEED", "11")))
nl = len(hidden) + 1
for k in range(1, nsteps + 1):
    idx = g.choice(len(rb), size=B, replace=False).astype(np.int32)
    et = g.standard_normal((B, act)).astype(np.float32)
    ea = g.standard_normal((B, act)).astype(np.float32)
    pre_pi = {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets["pi"].state_dict().items()}
    m_pre = np_(eng.adam_views("pi")[0][0]).astype(np.float64)
    alpha = float(eng.alpha_state.cpu().numpy()[1])
    eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
              eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, act))
    torch.cuda.synchronize()
    m_post = np_(eng.adam_views("pi")[0][0]).astype(np.float64)
    g_eng = (m_post - 0.9 * m_pre) / 0.1
    # float64 actor gradient through the engine's post-step critics
    W0 = pre_pi["net.0.weight"].clone().requires_grad_(True)
    sd = dict(pre_pi)
    sd["net.0.weight"] = W0
    s = torch.tensor(rows["obs"][idx], dtype=d)
    h = mlp64(sd, s, nl)
    mu, ls = h[:, :act], torch.clamp(h[:, act:], -20.0, 2.0)
    sdv = ls.exp()
    z = mu + torch.tensor(ea, dtype=d) * sdv
    a = torch.tanh(z)
    lp = (-((z - mu) ** 2) / (2 * sdv * sdv) - ls - 0.5 * np.log(2 * np.pi)).sum(1)
    lp = lp - (2 * (np.log(2) - z - F.softplus(-2 * z))).sum(1)
    qs = []
    for key in ("q1", "q2"):
        qsd = {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets[key].state_dict().items()}
        qs.append(mlp64(qsd, torch.cat([s, a], 1), nl)[:, 0])
    loss = (alpha * lp - torch.minimum(qs[0], qs[1])).mean()
    loss.backward()
    g64 = W0.grad.numpy()
    err = np.abs(g_eng - g64)
    scale = np.abs(g64).max() + 1e-30
    print(f"step {k}: |g64| max {scale:.3e} mean {np.abs(g64).mean():.3e}; |g_eng - g64| max {err.max():.3e}"
          f" mean {err.mean():.3e}; rel max {err.max() / scale:.2e}", flush=True)
    rel = err / scale
    N, K = rel.shape
    tiles = [(n0, k0, rel[n0:n0 + 32, k0:k0 + 32].max()) for n0 in range(0, N, 32) for k0 in range(0, K, 32)]
    bad = [t for t in tiles if t[2] > 1e-4]
    print(f"   tiles over 1e-4 rel: {len(bad)}/{len(tiles)} " + " ".join(f"({n0},{k0}):{r:.1e}" for n0, k0, r in bad[:20]))
    rmax = rel.max(1)
    print("   worst rows:", [(int(i), f"{rmax[i]:.1e}") for i in np.argsort(-rmax)[:8]])
    cmax = rel.max(0)
    print("   worst cols:", [(int(i), f"{cmax[i]:.1e}") for i in np.argsort(-cmax)[:8]])
    # inputs: relu boundary crossings of the actor rows' layer-0 pre-activations near 0
    pre0 = (s @ pre_pi["net.0.weight"].T + pre_pi["net.0.bias"]).numpy()
    print(f"   |pre0| min {np.abs(pre0).min():.2e}; entries under 1e-6: {(np.abs(pre0) < 1e-6).sum()}", flush=True)

# ---- which discrete choice of which batch row explains the difference?  For
# the last step: flip the min-Q choice of the rows with the smallest |q1 - q2|
# (float64), and report the rows nearest the log-std clamp, then compare each
# variant's gradient with the engine's.
if os.environ.get("DBG_FLIP"):
    qa, qb = qs[0].detach(), qs[1].detach()
    gap = (qa - qb).abs().numpy()
    order = np.argsort(gap)[:6]
    raw = h[:, act:].detach().numpy()
    print("   smallest |q1 - q2|:", [(int(r), f"{gap[r]:.2e}", f"q {qa[r].item():.4f}") for r in order])
    print("   log-std raw nearest the clamp [-20, 2]:", sorted(((float(min(abs(v - 2.0), abs(v + 20.0))), i) for i, v in
                                                              enumerate(raw.ravel())))[:4])
    for r in order:
        W0b = pre_pi["net.0.weight"].clone().requires_grad_(True)
        sd2 = dict(pre_pi)
        sd2["net.0.weight"] = W0b
        h2 = mlp64(sd2, s, nl)
        mu2, ls2 = h2[:, :act], torch.clamp(h2[:, act:], -20.0, 2.0)
        sd_2 = ls2.exp()
        z2 = mu2 + torch.tensor(ea, dtype=d) * sd_2
        a2 = torch.tanh(z2)
        lp2 = (-((z2 - mu2) ** 2) / (2 * sd_2 * sd_2) - ls2 - 0.5 * np.log(2 * np.pi)).sum(1)
        lp2 = lp2 - (2 * (np.log(2) - z2 - F.softplus(-2 * z2))).sum(1)
        q2s = []
        for key in ("q1", "q2"):
            qsd = {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets[key].state_dict().items()}
            q2s.append(mlp64(qsd, torch.cat([s, a2], 1), nl)[:, 0])
        mq = torch.minimum(q2s[0], q2s[1])
        flip = torch.maximum(q2s[0], q2s[1])
        sel = torch.zeros(B, dtype=torch.bool)
        sel[int(r)] = True
        mq = torch.where(sel, flip, mq)
        (alpha * lp2 - mq).mean().backward()
        e2 = np.abs(g_eng - W0b.grad.numpy()).max() / scale
        print(f"   flip min-Q of row {int(r)}: rel max vs engine {e2:.2e}", flush=True)
    # a single batch row r whose gradient differs gives G = g_eng - g64 =
    # delta_r (outer) s_r: rank one, its column factor parallel to s_r
    G = g_eng - g64
    u_, sv, vt = np.linalg.svd(G)
    v1 = vt[0]
    S = rows["obs"][idx].astype(np.float64)
    cos = np.abs(S @ v1) / (np.linalg.norm(S, axis=1) * np.linalg.norm(v1) + 1e-30)
    best = np.argsort(-cos)[:3]
    print(f"   G singular values {sv[:4]}; rows most parallel to its column factor:",
          [(int(r), f"{cos[r]:.4f}") for r in best], flush=True)
    r = int(best[0])
    hh = h.detach().numpy()[r]
    print(f"   row {r}: mu {hh[:act]}, log-std raw {hh[act:]}, z {z.detach().numpy()[r]}, a {a.detach().numpy()[r]},"
          f" q1 {qs[0][r].item():.6f} q2 {qs[1][r].item():.6f}, lp {lp[r].item():.6f}", flush=True)
    # pre-activations near 0 for that row: pi hidden layers and both critics' hidden layers
    def pre_acts(sd_, x, n):
        out = []
        for i in range(n - 1):
            x = x @ sd_[f"net.{2 * i}.weight"].T + sd_[f"net.{2 * i}.bias"]
            out.append(x.detach().numpy())
            x = torch.relu(x)
        return out
    for name, sd_, x in (("pi", pre_pi, s[r:r + 1]),
                         ("q1", {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets["q1"].state_dict().items()},
                          torch.cat([s, a], 1)[r:r + 1]),
                         ("q2", {kk: torch.tensor(np_(v), dtype=d) for kk, v in eng.nets["q2"].state_dict().items()},
                          torch.cat([s, a], 1)[r:r + 1])):
        for li, p in enumerate(pre_acts(sd_, x, nl)):
            print(f"   row {r} {name} layer {li}: |pre| min {np.abs(p).min():.3e} (unit {int(np.abs(p).argmin())})")
    eng_lp = eng.last_log_pi().cpu().numpy()
    print(f"   engine log pi of row {r}: {eng_lp[r]:.6f} (f64 {lp[r].item():.6f}); max |lp diff| {np.abs(eng_lp - lp.detach().numpy()).max():.2e} at row {int(np.abs(eng_lp - lp.detach().numpy()).argmax())}", flush=True)
