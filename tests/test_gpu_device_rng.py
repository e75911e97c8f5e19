"""The default (device-RNG) training path end to end, against the oracle.

The drop-in agent and bench.py train with ``train.rng: device``: the fused step
draws its replay indices from the Philox-keyed Feistel sampler and its two
rsample eps draws (target: agent.py:204, actor: agent.py:241; models.py:79-87)
from Philox4x32-10 + Box-Muller (sac_device.h philox_normal2).  Both are
restated in oracle/sampler_oracle.py.  These tests pin that path:

  * the device eps equal the host export and the oracle restatement (within 2
    ulps: the device's log / sin / cos are ocml's, the oracle's numpy's);
  * the draws are standard normal (moments, tails, KS) and independent
    (target vs actor draw, step vs step, row vs row, the two Box-Muller
    outputs of one counter) over ~1e6 draws;
  * device-RNG steps (eager and graph-replayed, staged next-step batches
    included) equal the oracle fed the restated indices AND eps, at the fp32
    tolerances of tests/test_gpu_parity.py;
  * a 200-step C2 fp32 run with injected inputs stays on the oracle: the
    losses within 1e-5 rel over the first 50 steps and 1e-3 rel over all 200,
    and the parameters within the drift bounds written in the test.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import sac_oracle as O
from oracle import sampler_oracle as S

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
NET_KEYS = {"policy": "pi", "q1": "q1", "q2": "q2", "q1t": "q1t", "q2t": "q2t"}


@pytest.fixture(scope="module")
def lib():
    from sac import _engine as E

    lb = E.load_library()
    lb.sac_debug_eps_host.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p]
    lb.sac_debug_eps_device.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p]
    return lb


def device_eps(lib, seed, step, B, A):
    from sac import _engine as E

    out = torch.empty(2, B, A, dtype=torch.float32, device=DEV)
    E.check(lib.sac_debug_eps_device(seed, step, B, A, E.ptr(out), E.stream_handle(DEV)))
    return out


def host_eps(lib, seed, step, B, A):
    out = np.zeros((2, B, A), np.float32)
    assert lib.sac_debug_eps_host(seed, step, B, A, out.ctypes.data) == 0
    return out


# ---------------------------------------------------------------- the generator
@pytest.mark.parametrize("seed,step,B,A", [(0, 0, 256, 4), (3, 17, 4096, 4), (7, 2**33 + 5, 300, 1),
                                           (2**40 + 1, 999, 64, 3), (11, 5, 256, 2)])
def test_device_eps_equal_host_and_oracle(lib, seed, step, B, A):
    dev = device_eps(lib, seed, step, B, A).cpu().numpy()
    host = host_eps(lib, seed, step, B, A)
    ora = S.eps_draws(seed, step, B, A)
    # ocml vs glibc vs numpy float32 log/sin/cos: at most a couple of ulps
    np.testing.assert_allclose(dev, host, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dev, ora, rtol=1e-6, atol=1e-6)
    assert np.mean(dev == host) > 0.5  # mostly bit-equal: the same Philox words and the same fp32 formula


def _phi(x):
    from scipy.special import ndtr

    return ndtr(x)


def test_device_eps_are_standard_normal_and_independent(lib):
    """~1e6 draws per step (B = 131,072 rows x 4 dims x 2 draws), two steps.
    Every bound is 5 standard errors of the statistic under iid N(0, 1)."""
    from scipy import stats

    B, A, seed = 131_072, 4, 5
    e0 = device_eps(lib, seed, 40, B, A).double().cpu().numpy()  # [2][B][A]
    e1 = device_eps(lib, seed, 41, B, A).double().cpu().numpy()
    x = np.concatenate([e0.ravel(), e1.ravel()])
    n = x.size
    assert n >= 2_000_000
    assert np.all(np.isfinite(x))
    # Box-Muller on 24-bit uniforms: |eps| <= sqrt(2 * 24 ln 2) = 5.77
    assert np.abs(x).max() <= 5.77
    m, v = x.mean(), x.var()
    assert abs(m) < 5 / np.sqrt(n), m
    assert abs(v - 1) < 5 * np.sqrt(2 / n), v
    sk, ku = stats.skew(x), stats.kurtosis(x, fisher=False)
    assert abs(sk) < 5 * np.sqrt(6 / n), sk
    assert abs(ku - 3) < 5 * np.sqrt(24 / n), ku
    for t in (1.0, 2.0, 3.0, 4.0):  # two-sided tail frequencies
        p = 2 * (1 - _phi(t))
        got = np.mean(np.abs(x) > t)
        assert abs(got - p) < 5 * np.sqrt(p * (1 - p) / n) + 1e-7, (t, got, p)
    ks = stats.kstest(x[::4], "norm")  # every 4th draw: 5e5 samples
    assert ks.pvalue > 1e-4, ks
    # independence: correlations between streams that must not share a draw
    pairs = {
        "target vs actor draw (same step, row, dim)": (e0[0], e0[1]),
        "step t vs t+1 (same draw, row, dim)": (e0[0], e1[0]),
        "row b vs b+1": (e0[0][:-1], e0[0][1:]),
        "Box-Muller cos vs sin output (dims 2p, 2p+1)": (e0[0][:, 0::2], e0[0][:, 1::2]),
        "dim 0 vs dim 2 (next counter pair)": (e0[1][:, 0], e0[1][:, 2]),
    }
    for name, (a, b) in pairs.items():
        r = np.corrcoef(a.ravel(), b.ravel())[0, 1]
        assert abs(r) < 5 / np.sqrt(a.size), (name, r)
    # joint uniformity of (target, actor) in 10 x 10 probability bins: chi-square, dof 99
    u = np.floor(_phi(e0[0].ravel()) * 10).clip(0, 9).astype(int)
    w = np.floor(_phi(e0[1].ravel()) * 10).clip(0, 9).astype(int)
    h = np.bincount(u * 10 + w, minlength=100).astype(float)
    exp = h.sum() / 100
    chi = ((h - exp) ** 2 / exp).sum()
    assert chi < 99 + 5 * np.sqrt(2 * 99), chi


# ---------------------------------------------------------------- the step on the device RNG
def _engine(cfgname, precision, seed, capacity):
    import bench

    c = dict(bench.CONFIGS[cfgname])
    bench.CONFIGS[cfgname] = dict(c, capacity=capacity)
    try:
        return bench.build_engine(cfgname, precision, seed, DEV)
    finally:
        bench.CONFIGS[cfgname] = c


def _oracle_for(eng, A):
    sds = {k: {kk: v.detach().cpu().numpy().copy() for kk, v in m.state_dict().items()} for k, m in eng.nets.items()}
    hp = O.SacHyper(alpha=0.1, auto_entropy_tuning=True)  # bench.build_engine's hyper-parameters
    st = O.SacState.fresh(O.MLP.from_state_dict(sds["pi"], "relu"), O.MLP.from_state_dict(sds["q1"], "relu"),
                          O.MLP.from_state_dict(sds["q2"], "relu"), hp, A)
    return st, hp


def _rows(rb):
    return {k: getattr(rb, k).cpu().numpy() for k in ("obs", "act", "rew", "next_obs", "done")}


def _batch(rows, idx):
    return O.Batch(rows["obs"][idx], rows["act"][idx], rows["rew"][idx], rows["next_obs"][idx], rows["done"][idx])


def _check_losses(got, ref, st, tag, rtol=1e-4):
    floor = float(np.mean(np.abs(st.alpha * ref["log_pi"])) + np.mean(np.abs(ref["y"]))) + 1e-6
    for i, (g, w) in enumerate(zip(got, ref["losses"])):
        f = floor if i == 2 else 1e-3
        assert abs(g - w) <= rtol * max(abs(w), f), (tag, i, g, w)


def _check_params(eng, st, hp, k, tag):
    """tests/test_gpu_parity.py's fp32 bar: max error within 2 lr per step of
    Adam movement (targets: tau times that, accumulated) and 99.5% of the
    elements within 1e-6."""
    lrs = {"policy": hp.actor_lr, "q1": hp.critic_lr, "q2": hp.critic_lr, "q1t": hp.critic_lr * hp.tau,
           "q2t": hp.critic_lr * hp.tau}
    nets = {"policy": st.pi, "q1": st.q1, "q2": st.q2, "q1t": st.q1t, "q2t": st.q2t}
    for key, ek in NET_KEYS.items():
        mine = {kk: v.detach().cpu().numpy() for kk, v in eng.nets[ek].state_dict().items()}
        lr = lrs[key] * (k if key in ("policy", "q1", "q2") else k * (k + 1) / 2)
        for pk, want in nets[key].state_dict().items():
            d = np.abs(mine[pk] - want)
            assert d.max() <= 2 * lr + 1e-5, (tag, key, pk, d.max())
            assert np.mean(d <= 1e-6) >= 0.995, (tag, key, pk, np.mean(d <= 1e-6))
    la = float(eng.alpha_state[0].item())
    assert abs(la - st.log_alpha) <= 1e-7, (tag, la, st.log_alpha)


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_device_rng_steps_match_oracle(lib, cfg):
    """Device-sampled indices and device eps (indices=None, eps=None): three
    eager steps, each checked against the oracle fed sampler_oracle's indices
    and eps for (seed, rng_step), then three more replayed from one hipGraph
    (phase C stages each next step's batch) checked at the end.  C2 fp32 (the
    headline configuration, 1e6-row sized replay cut to 5,000 rows so the
    oracle can index it) and C4."""
    seed = 3
    eng, rb, c = _engine(cfg, "fp32", seed, 5000)
    assert int(eng.cfg.seed) == seed
    B, A = c["batch"], c["act"]
    st, hp = _oracle_for(eng, A)
    rows = _rows(rb)

    def oracle_step():
        t = int(eng.rng_step.item())
        idx = np.asarray(S.sample_indices(len(rb), B, seed, t), np.int64)
        e = S.eps_draws(seed, t, B, A)
        return O.training_step(st, hp, _batch(rows, idx), e[0], e[1])

    for k in range(1, 4):
        ref = oracle_step()
        eng.train(rb, 1)  # device sampler + device eps
        torch.cuda.synchronize()
        _check_losses(eng.losses(), ref, st, (cfg, k))
        np.testing.assert_allclose(eng.last_targets().cpu().numpy(), ref["y"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(eng.last_log_pi().cpu().numpy(), ref["log_pi"], rtol=1e-4, atol=1e-4)
        _check_params(eng, st, hp, k, (cfg, k))
    t0 = int(eng.rng_step.item())
    for j in range(3):  # the oracle walks the same three steps
        idx = np.asarray(S.sample_indices(len(rb), B, seed, t0 + j), np.int64)
        e = S.eps_draws(seed, t0 + j, B, A)
        ref = O.training_step(st, hp, _batch(rows, idx), e[0], e[1])
    eng.train_graph(rb, 3, chunk=3)
    torch.cuda.synchronize()
    eng.check()
    assert int(eng.rng_step.item()) == t0 + 3
    _check_losses(eng.losses(), ref, st, (cfg, "graph"))
    _check_params(eng, st, hp, 6, (cfg, "graph"))


def test_c2_200_steps_stay_on_the_oracle():
    """C2 fp32, 200 consecutive steps with injected indices and eps (seeded
    numpy draws), engine and oracle stepping side by side from the same state.

    The two differ only in fp32 summation order, which Adam amplifies: an
    element whose gradient is ~0 can take a +lr step on one side and -lr on the
    other, so the two trajectories separate slowly (measured on MI355X: loss
    deviations <= 1.2e-7 rel through step 50, 5e-5 at step 100, 5.2e-4 at step
    200; y 3e-7 through step 20, 2.7e-3 at step 200).  Bounds (written here):
      * losses: the north-star bar, 1e-3 rel, at EVERY step (L_pi with the abs
        floor of tests/test_gpu_parity.py), and 1e-5 rel over the first 50;
      * y: |dy| <= 1e-5 (1 + |y|) over the first 20 steps, 1e-4 over the
        first 50, 1e-2 (1 + |y|) at every step (y also carries the target
        networks' accumulated drift; since phase B sums the critics' output
        bias gradient from the seeded columns, y reaches ~2e-5 by step 50);
      * after 200 steps every online parameter within 2 lr k of the oracle
        (the Adam movement bound) with a mean |error| within 0.01 lr k; the
        target networks (tau-averages of k online states) within 2 lr tau
        k(k+1)/2 with a mean within 0.005 of it; log alpha within 1e-6.
    The measured per-step deviations are printed (run with -s)."""
    seed, k_total = 0, 200
    eng, rb, c = _engine("c2", "fp32", seed, 20_000)
    B, A = c["batch"], c["act"]
    st, hp = _oracle_for(eng, A)
    rows = _rows(rb)
    g = np.random.default_rng(2024)
    dev = np.zeros((k_total, 5))  # rel dev of the 4 losses, then max |dy| / (1 + |y|)
    for k in range(1, k_total + 1):
        idx = g.choice(len(rb), size=B, replace=False).astype(np.int32)
        et = g.standard_normal((B, A)).astype(np.float32)
        ea = g.standard_normal((B, A)).astype(np.float32)
        ref = O.training_step(st, hp, _batch(rows, idx), et, ea)
        eng.train(rb, 1, indices=torch.from_numpy(idx).reshape(1, B),
                  eps=torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, A))
        got = eng.losses()
        floor = float(np.mean(np.abs(st.alpha * ref["log_pi"])) + np.mean(np.abs(ref["y"]))) + 1e-6
        for i in range(4):
            f = floor if i == 2 else 1e-3
            dev[k - 1, i] = abs(got[i] - ref["losses"][i]) / max(abs(ref["losses"][i]), f)
        y = eng.last_targets().cpu().numpy()
        dev[k - 1, 4] = float(np.max(np.abs(y - ref["y"]) / (1.0 + np.abs(ref["y"]))))
    kk = k_total * (k_total + 1) / 2  # targets: tau times the accumulated online error
    lrs = {"policy": hp.actor_lr * k_total, "q1": hp.critic_lr * k_total, "q2": hp.critic_lr * k_total,
           "q1t": hp.critic_lr * hp.tau * kk, "q2t": hp.critic_lr * hp.tau * kk}
    nets = {"policy": st.pi, "q1": st.q1, "q2": st.q2, "q1t": st.q1t, "q2t": st.q2t}
    report = {}
    for key, ek in NET_KEYS.items():
        lr_k = lrs[key]
        mine = {kk: v.detach().cpu().numpy() for kk, v in eng.nets[ek].state_dict().items()}
        d = np.concatenate([np.abs(mine[pk] - w).ravel() for pk, w in nets[key].state_dict().items()])
        report[key] = {"max/lr_k": float(d.max() / lr_k), "mean/lr_k": float(d.mean() / lr_k),
                       "frac<=1e-6": float(np.mean(d <= 1e-6))}
    la = float(eng.alpha_state[0].item())
    summary = {"loss_rel_dev_max": dev[:, :4].max(0).tolist(), "loss_rel_dev_max_first50": dev[:50, :4].max(0).tolist(),
               "y_dev_max": float(dev[:, 4].max()), "y_dev_max_first50": float(dev[:50, 4].max()),
               "loss_rel_dev_at": {str(k): dev[k - 1, :4].tolist() for k in (1, 10, 50, 100, 150, 200)},
               "params": report, "log_alpha_err": abs(la - st.log_alpha)}
    print("\n200-step C2 fp32 drift vs oracle:", summary)
    assert dev[:, :4].max() <= 1e-3, summary
    assert dev[:50, :4].max() <= 1e-5, summary
    assert dev[:20, 4].max() <= 1e-5 and dev[:50, 4].max() <= 1e-4 and dev[:, 4].max() <= 1e-2, summary
    for key in NET_KEYS:
        assert report[key]["max/lr_k"] <= 2.0 + 1e-5 / lrs[key], (key, summary)
        assert report[key]["mean/lr_k"] <= (0.01 if key in ("policy", "q1", "q2") else 0.005), (key, summary)
    assert abs(la - st.log_alpha) <= 1e-6, summary
