"""CPU ORACLE for the SAC gradient step — TEST INFRASTRUCTURE ONLY.

This module is the parity checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``soft-actor-critic_amd/sac`` -> ``libsac_engine.so``) never
calls into it and fails loudly when the HIP library is missing.

It is a plain-numpy float32 restatement of the reference algorithm, op for op:

* replay storage + uniform sampling without replacement
      reference sac/replay_buffer.py:11-42  (deque(maxlen) + random.sample)
* batch tensorisation                       sac/agent.py:166-193
* MLP (Linear/activation stack)             sac/models.py:104-149
* Q(s,a) = MLP(cat[s,a]).squeeze(-1)        sac/models.py:30-33
* squashed Gaussian policy head             sac/models.py:73-87
      (torch.distributions.Normal.rsample / log_prob, softplus threshold 20)
* target y = r + g(1-d)(min Qt - a logpi')  sac/agent.py:195-211
* critic MSE + Adam                         sac/agent.py:213-236
* actor loss mean(a logpi - min Q) + Adam   sac/agent.py:238-260
* alpha loss on float64 log_alpha + Adam    sac/agent.py:263-280, 43-53
* Polyak t = tau p + (1 - tau) t            sac/agent.py:282-300
* Adam single-tensor math (torch/optim/adam.py, lerp / mul+addcmul / addcdiv)

Backward passes are written out by hand (the reference relies on autograd); the
derivative of each op follows torch's registered formula (threshold_backward,
elu_backward, gelu_backward, softplus_backward, tanh_backward, clamp_backward,
``minimum`` ties split 1/2-1/2, mse_loss_backward = 2(x-y)/N).

Parity of this restatement is pinned by ``tests/golden/*.npz``, captured from the
reference itself (``tests/golden/make_golden.py``) and checked by
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
import random
from collections import deque, namedtuple
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

F32 = np.float32

# ----------------------------------------------------------------------------- activations
_SELU_SCALE = F32(1.0507009873554804934193349852946)
_SELU_ALPHA = F32(1.6732632423543772848170429916717)
_LEAKY = F32(0.01)


def _erf(x: np.ndarray) -> np.ndarray:
    from scipy.special import erf  # scipy is present in the image

    return erf(x.astype(np.float64)).astype(F32)


def act_fwd(name: str, p: np.ndarray) -> np.ndarray:
    """Forward of reference sac/models.py:104-112 ``_ACTIVATIONS``."""
    if name == "identity":
        return p
    if name == "relu":
        return np.maximum(p, F32(0))
    if name == "tanh":
        return np.tanh(p)
    if name == "elu":
        return np.where(p > 0, p, np.expm1(p)).astype(F32)
    if name == "leaky_relu":
        return np.where(p > 0, p, p * _LEAKY).astype(F32)
    if name == "gelu":
        return (p * F32(0.5) * (F32(1) + _erf(p * F32(1 / math.sqrt(2))))).astype(F32)
    if name == "selu":
        return (_SELU_SCALE * np.where(p > 0, p, _SELU_ALPHA * np.expm1(p))).astype(F32)
    raise KeyError(name)


def act_bwd(name: str, p: np.ndarray, h: np.ndarray, g: np.ndarray) -> np.ndarray:
    """d act / d p applied to upstream grad g (torch *_backward formulas)."""
    if name == "identity":
        return g
    if name == "relu":  # threshold_backward(grad, result, 0)
        return np.where(h > 0, g, F32(0)).astype(F32)
    if name == "tanh":  # tanh_backward(grad, result)
        return (g * (F32(1) - h * h)).astype(F32)
    if name == "elu":  # elu_backward(is_result=False): x<=0 -> g*exp(x)
        return np.where(p > 0, g, g * np.exp(p)).astype(F32)
    if name == "leaky_relu":
        return np.where(p > 0, g, g * _LEAKY).astype(F32)
    if name == "gelu":
        cdf = F32(0.5) * (F32(1) + _erf(p * F32(1 / math.sqrt(2))))
        pdf = np.exp(F32(-0.5) * p * p) * F32(1 / math.sqrt(2 * math.pi))
        return (g * (cdf + p * pdf)).astype(F32)
    if name == "selu":
        return np.where(p > 0, g * _SELU_SCALE, g * _SELU_SCALE * _SELU_ALPHA * np.exp(p)).astype(F32)
    raise KeyError(name)


def softplus(x: np.ndarray) -> np.ndarray:
    """torch softplus(beta=1, threshold=20)."""
    return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, F32(20))))).astype(F32)


def softplus_grad(x: np.ndarray) -> np.ndarray:
    z = np.exp(np.minimum(x, F32(20)))
    return np.where(x > 20, F32(1), z / (z + F32(1))).astype(F32)


# ----------------------------------------------------------------------------- MLP
@dataclass
class MLP:
    """Linear stack of reference build_mlp (sac/models.py:115-149).

    ``W[i]`` is [out, in] (nn.Linear layout), ``b[i]`` is [out]."""

    W: List[np.ndarray]
    b: List[np.ndarray]
    hidden_act: str = "relu"
    out_act: str = "identity"

    def copy(self) -> "MLP":
        return MLP([w.copy() for w in self.W], [x.copy() for x in self.b], self.hidden_act, self.out_act)

    def params(self) -> List[np.ndarray]:
        out = []
        for w, b in zip(self.W, self.b):
            out += [w, b]
        return out

    def state_dict(self) -> Dict[str, np.ndarray]:
        sd = {}
        for i, (w, b) in enumerate(zip(self.W, self.b)):
            sd[f"net.{2 * i}.weight"] = w
            sd[f"net.{2 * i}.bias"] = b
        return sd

    @staticmethod
    def from_state_dict(sd: Dict[str, np.ndarray], hidden_act="relu", out_act="identity") -> "MLP":
        n = len([k for k in sd if k.endswith(".weight")])
        W = [np.asarray(sd[f"net.{2 * i}.weight"], F32).copy() for i in range(n)]
        b = [np.asarray(sd[f"net.{2 * i}.bias"], F32).copy() for i in range(n)]
        return MLP(W, b, hidden_act, out_act)

    def forward(self, x: np.ndarray):
        """Returns output and the per-layer cache [(input, pre, post)]."""
        cache = []
        h = x.astype(F32)
        n = len(self.W)
        for i in range(n):
            p = (h @ self.W[i].T + self.b[i]).astype(F32)
            act = self.hidden_act if i < n - 1 else self.out_act
            o = act_fwd(act, p)
            cache.append((h, p, o))
            h = o
        return h, cache

    def backward(self, cache, g_out: np.ndarray, need_dx: bool = False):
        """Grads of every W, b given d(out); optionally d(input)."""
        n = len(self.W)
        gW: List[Optional[np.ndarray]] = [None] * n
        gb: List[Optional[np.ndarray]] = [None] * n
        g = g_out.astype(F32)
        dx = None
        for i in reversed(range(n)):
            h_in, p, o = cache[i]
            act = self.hidden_act if i < n - 1 else self.out_act
            gp = act_bwd(act, p, o, g)
            gW[i] = (gp.T @ h_in).astype(F32)
            gb[i] = gp.sum(0, dtype=F32)
            if i > 0 or need_dx:
                g = (gp @ self.W[i]).astype(F32)
        if need_dx:
            dx = g
        return gW, gb, dx


def q_forward(q: MLP, s, a):
    out, cache = q.forward(np.concatenate([s, a], axis=-1))
    return out[:, 0], cache


# ----------------------------------------------------------------------------- policy head
@dataclass
class PolicyCfg:
    log_std_min: float = -20.0
    log_std_max: float = 2.0
    action_scale: float = 1.0


_LOG2 = F32(math.log(2.0))
_HALF_LOG_2PI = F32(math.log(math.sqrt(2 * math.pi)))


def policy_sample(pi: MLP, s: np.ndarray, eps: np.ndarray, pc: PolicyCfg):
    """PolicyNetwork.sample_action with injected eps (sac/models.py:79-87)."""
    out, cache = pi.forward(s)
    A = out.shape[1] // 2
    mu, log_std = out[:, :A], out[:, A:]
    ls = np.clip(log_std, F32(pc.log_std_min), F32(pc.log_std_max))
    std = np.exp(ls).astype(F32)
    z = (mu + eps * std).astype(F32)
    t = np.tanh(z).astype(F32)
    a = (t * F32(pc.action_scale)).astype(F32)
    diff = z - mu
    var = std * std
    lp = (-(diff * diff) / (F32(2) * var) - np.log(std) - _HALF_LOG_2PI).astype(F32)
    corr = (F32(2) * (_LOG2 - z - softplus(F32(-2) * z))).astype(F32)
    logpi = (lp.sum(-1, dtype=F32) - corr.sum(-1, dtype=F32)).astype(F32)
    ctx = dict(cache=cache, mu=mu, log_std=log_std, std=std, z=z, t=t, eps=eps, diff=diff, var=var)
    return a, logpi, ctx


def policy_sample_backward(pi: MLP, ctx, g_a: np.ndarray, g_logpi: np.ndarray, pc: PolicyCfg):
    """Hand-written autograd of ``policy_sample`` w.r.t. the MLP output."""
    std, z, t, eps, diff, var = ctx["std"], ctx["z"], ctx["t"], ctx["eps"], ctx["diff"], ctx["var"]
    gl = g_logpi[:, None].astype(F32)
    # a = tanh(z) * scale
    g_z = (g_a * F32(pc.action_scale)) * (F32(1) - t * t)
    # -corr: corr = 2*(log2 - z - softplus(-2z))
    g_corr = -gl
    g_z = g_z + g_corr * F32(2) * (F32(-1) + F32(2) * softplus_grad(F32(-2) * z))
    # lp = -(diff^2)/(2 var) - log(std) - c
    two_var = F32(2) * var
    g_sq = -gl / two_var
    g_twovar = gl * (diff * diff) / (two_var * two_var)
    g_var = F32(2) * g_twovar
    g_std = F32(2) * std * g_var - gl / std
    g_diff = F32(2) * diff * g_sq
    g_z = g_z + g_diff
    g_mu = -g_diff
    # z = mu + eps*std
    g_mu = g_mu + g_z
    g_std = g_std + g_z * eps
    g_ls = g_std * std
    ls_raw = ctx["log_std"]
    in_range = (ls_raw >= F32(pc.log_std_min)) & (ls_raw <= F32(pc.log_std_max))
    g_logstd = np.where(in_range, g_ls, F32(0)).astype(F32)
    return np.concatenate([g_mu, g_logstd], axis=1).astype(F32)


# ----------------------------------------------------------------------------- optimizer
@dataclass
class AdamState:
    m: List[np.ndarray]
    v: List[np.ndarray]
    step: float = 0.0

    @staticmethod
    def zeros_like(params: List[np.ndarray]) -> "AdamState":
        return AdamState([np.zeros_like(p) for p in params], [np.zeros_like(p) for p in params], 0.0)


def adam_update(params, grads, st: AdamState, lr: float, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor path (adam.py _single_tensor_adam)."""
    st.step += 1.0
    bc1 = 1.0 - beta1 ** st.step
    bc2 = 1.0 - beta2 ** st.step
    step_size = lr / bc1
    bc2_sqrt = math.sqrt(bc2)
    dt = params[0].dtype
    w = dt.type(1.0 - beta1)
    for i, (p, g) in enumerate(zip(params, grads)):
        m, v = st.m[i], st.v[i]
        m[...] = m + w * (g - m)  # lerp, weight < 0.5
        v[...] = v * dt.type(beta2) + dt.type(1.0 - beta2) * g * g
        denom = np.sqrt(v) / dt.type(bc2_sqrt) + dt.type(eps)
        p[...] = p + dt.type(-step_size) * m / denom


# ----------------------------------------------------------------------------- agent state
@dataclass
class SacHyper:
    gamma: float = 0.99
    tau: float = 0.005
    alpha: float = 0.1
    auto_entropy_tuning: bool = False
    actor_lr: float = 3e-4
    critic_lr: float = 3e-4
    alpha_lr: float = 3e-4
    policy: PolicyCfg = field(default_factory=PolicyCfg)

    @staticmethod
    def from_config(cfg: dict) -> "SacHyper":
        s, p = cfg["sac"], cfg["policy_net"]
        return SacHyper(
            gamma=s["gamma"], tau=s["tau"], alpha=s["alpha"],
            auto_entropy_tuning=bool(s["auto_entropy_tuning"]),
            actor_lr=s["actor_lr"], critic_lr=s["critic_lr"], alpha_lr=s["alpha_lr"],
            policy=PolicyCfg(p["log_std_min"], p["log_std_max"], p["action_scale"]),
        )


@dataclass
class SacState:
    pi: MLP
    q1: MLP
    q2: MLP
    q1t: MLP
    q2t: MLP
    opt_pi: AdamState
    opt_q1: AdamState
    opt_q2: AdamState
    act_dim: int
    log_alpha: Optional[float] = None  # float64 when auto tuning
    alpha: float = 0.1                 # value as the reference holds it (fp64 or fp32)
    opt_alpha_m: float = 0.0
    opt_alpha_v: float = 0.0
    opt_alpha_step: float = 0.0
    # True after the reference's load_agent with auto-tuning: log_alpha is the
    # checkpoint's tensor while alpha_optimizer still holds the old one
    # (sac/agent.py:550-554), so L_alpha is computed but nothing updates alpha
    alpha_orphaned: bool = False

    @staticmethod
    def fresh(pi: MLP, q1: MLP, q2: MLP, hp: SacHyper, act_dim: int) -> "SacState":
        st = SacState(pi, q1, q2, q1.copy(), q2.copy(),
                      AdamState.zeros_like(pi.params()), AdamState.zeros_like(q1.params()),
                      AdamState.zeros_like(q2.params()), act_dim)
        if hp.auto_entropy_tuning:
            st.log_alpha = float(np.log(hp.alpha))
            st.alpha = math.exp(st.log_alpha)
        else:
            st.alpha = float(F32(hp.alpha))  # torch.tensor(alpha) is fp32 (agent.py:55)
        return st


Batch = namedtuple("Batch", ("s", "a", "r", "s2", "d"))


def training_step(st: SacState, hp: SacHyper, batch: Batch, eps_t: np.ndarray, eps_a: np.ndarray):
    """One reference ``training_step`` (agent.py:302-327) on an injected batch.

    Mutates ``st`` in place; returns dict(losses=[Lq1, Lq2, Lpi, Lalpha], y, log_pi)."""
    s, a, r, s2, d = (np.asarray(x, F32) for x in batch)
    B = s.shape[0]
    alpha32 = F32(st.alpha)
    pc = hp.policy

    # ---- target (agent.py:195-211), pre-update pi and target nets
    a2, lp2, _ = policy_sample(st.pi, s2, eps_t, pc)
    qt1, _ = q_forward(st.q1t, s2, a2)
    qt2, _ = q_forward(st.q2t, s2, a2)
    minq = np.minimum(qt1, qt2)
    y = (r + (F32(hp.gamma) * (F32(1) - d)) * (minq - alpha32 * lp2)).astype(F32)

    # ---- critics (agent.py:213-236)
    losses = []
    for q, opt in ((st.q1, st.opt_q1), (st.q2, st.opt_q2)):
        qv, cache = q_forward(q, s, a)
        diff = qv - y
        losses.append(float(np.mean(diff * diff, dtype=F32)))
        g_q = (F32(2.0 / B) * diff)[:, None].astype(F32)
        gW, gb, _ = q.backward(cache, g_q)
        grads = []
        for w_, b_ in zip(gW, gb):
            grads += [w_, b_]
        adam_update(q.params(), grads, opt, hp.critic_lr)

    # ---- actor (agent.py:238-260), post-update critics
    at, lp, ctx = policy_sample(st.pi, s, eps_a, pc)
    q1v, c1 = q_forward(st.q1, s, at)
    q2v, c2 = q_forward(st.q2, s, at)
    minq_a = np.minimum(q1v, q2v)
    lpi = float(np.mean(alpha32 * lp - minq_a, dtype=F32))
    losses.append(lpi)
    g_min = np.full(B, F32(-1.0 / B), F32)
    tie = q1v == q2v
    g1 = np.where(tie, g_min / F32(2), np.where(q1v < q2v, g_min, F32(0))).astype(F32)
    g2 = np.where(tie, g_min / F32(2), np.where(q2v < q1v, g_min, F32(0))).astype(F32)
    O = s.shape[1]
    _, _, dx1 = st.q1.backward(c1, g1[:, None], need_dx=True)
    _, _, dx2 = st.q2.backward(c2, g2[:, None], need_dx=True)
    g_a = (dx1[:, O:] + dx2[:, O:]).astype(F32)
    g_lp = np.full(B, alpha32 * F32(1.0 / B), F32)
    g_out = policy_sample_backward(st.pi, ctx, g_a, g_lp, pc)
    gW, gb, _ = st.pi.backward(ctx["cache"], g_out)
    grads = []
    for w_, b_ in zip(gW, gb):
        grads += [w_, b_]
    adam_update(st.pi.params(), grads, st.opt_pi, hp.actor_lr)

    # ---- alpha (agent.py:263-280), fp64 log_alpha, fp32 loss
    if hp.auto_entropy_tuning:
        H = F32(-float(st.act_dim))
        la32 = F32(st.log_alpha)
        term = (lp + H).astype(F32)
        losses.append(float(-np.mean(la32 * term, dtype=F32)))
    if hp.auto_entropy_tuning and not st.alpha_orphaned:
        g = float(np.sum(F32(-1.0 / B) * term, dtype=F32))
        st.opt_alpha_step += 1.0
        b1, b2, e = 0.9, 0.999, 1e-8
        st.opt_alpha_m = st.opt_alpha_m + (1 - b1) * (g - st.opt_alpha_m)
        st.opt_alpha_v = st.opt_alpha_v * b2 + (1 - b2) * g * g
        bc1 = 1 - b1 ** st.opt_alpha_step
        bc2 = 1 - b2 ** st.opt_alpha_step
        denom = math.sqrt(st.opt_alpha_v) / math.sqrt(bc2) + e
        st.log_alpha = st.log_alpha + (-hp.alpha_lr / bc1) * st.opt_alpha_m / denom
        st.alpha = math.exp(st.log_alpha)
    elif not hp.auto_entropy_tuning:
        losses.append(float("nan"))

    # ---- Polyak (agent.py:282-300)
    tau, omt = F32(hp.tau), F32(1.0 - hp.tau)
    for tgt, src in ((st.q1t, st.q1), (st.q2t, st.q2)):
        for tp, sp in zip(tgt.params(), src.params()):
            tp[...] = (tau * sp + omt * tp).astype(F32)

    return dict(losses=losses, y=y, log_pi=lp)


# ----------------------------------------------------------------------------- replay (sampling semantics)
Transition = namedtuple("Transition", ("state", "action", "reward", "next_state", "done"))


class ReplayDeque:
    """reference sac/replay_buffer.py:11-42: FIFO deque(maxlen), random.sample."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        self.memory: deque = deque(maxlen=capacity)

    def push(self, s, a, r, s2, d):
        self.memory.append(Transition(s, a, r, s2, d))

    def sample(self, batch_size: int):
        if len(self.memory) < batch_size:
            raise ValueError(f"Not enough samples in the replay buffer to sample {batch_size} transitions. "
                             f"Current size: {len(self.memory)}")
        return random.sample(self.memory, batch_size)

    def __len__(self):
        return len(self.memory)


def sample_batch(buf: ReplayDeque, batch_size: int) -> Batch:
    """agent.py:166-193 (stack + float32 conversion), host side."""
    tr = buf.sample(batch_size)
    cols = Transition(*zip(*tr))
    return Batch(np.stack(cols.state).astype(F32), np.stack(cols.action).astype(F32),
                 np.array(cols.reward, dtype=F32), np.stack(cols.next_state).astype(F32),
                 np.array(cols.done, dtype=F32))


# ----------------------------------------------------------------------------- fixture helpers
def state_from_fixture(fx, prefix: str, hp: SacHyper, cfg: dict, act_dim: int) -> SacState:
    def net(name, hidden_act):
        sd = {k.split("/", 2)[2]: fx[k] for k in fx.files if k.startswith(f"{prefix}/{name}/") and "#" not in k}
        return MLP.from_state_dict(sd, hidden_act, "identity")

    qa = cfg["q_net"]["hidden_layers_act"]
    pa = cfg["policy_net"]["hidden_layers_act"]
    qo = cfg["q_net"]["output_activation"]
    po = cfg["policy_net"]["output_activation"]
    pi, q1, q2 = net("policy", pa), net("q1", qa), net("q2", qa)
    pi.out_act, q1.out_act, q2.out_act = po, qo, qo
    st = SacState.fresh(pi, q1, q2, hp, act_dim)
    st.q1t, st.q2t = net("q1t", qa), net("q2t", qa)
    st.q1t.out_act = st.q2t.out_act = qo
    return st


# ----------------------------------------------------------------------------- checkpoints
def load_checkpoint(ckpt: dict, hp: SacHyper, act_dim: int, q_act: str = "relu", pi_act: str = "relu") -> SacState:
    """The reference's ``load_agent`` (sac/agent.py:538-554) on a checkpoint dict
    as ``save_agent`` writes it (agent.py:521-536; tensors as numpy arrays):
    five state_dicts, three torch Adam state_dicts, and with auto-tuning
    ``log_alpha`` + the alpha optimizer's state_dict.  The alpha optimizer state
    is loaded into an optimizer that no longer owns ``log_alpha``: the returned
    state has ``alpha_orphaned`` set and alpha = exp(log_alpha)."""
    def sd(key):
        return {k: np.asarray(v, F32) for k, v in ckpt[key].items()}

    st = SacState(MLP.from_state_dict(sd("policy_net_state_dict"), pi_act),
                  MLP.from_state_dict(sd("q_net1_state_dict"), q_act), MLP.from_state_dict(sd("q_net2_state_dict"), q_act),
                  MLP.from_state_dict(sd("q_net1_target_state_dict"), q_act),
                  MLP.from_state_dict(sd("q_net2_target_state_dict"), q_act), None, None, None, act_dim)
    for name, net in (("policy_optimizer_state_dict", st.pi), ("q1_optimizer_state_dict", st.q1),
                      ("q2_optimizer_state_dict", st.q2)):
        o = ckpt[name]["state"]
        ps = net.params()
        ad = AdamState.zeros_like(ps)
        for i in range(len(ps)):
            if i in o:
                ad.m[i][...] = np.asarray(o[i]["exp_avg"], F32).reshape(ps[i].shape)
                ad.v[i][...] = np.asarray(o[i]["exp_avg_sq"], F32).reshape(ps[i].shape)
                ad.step = float(o[i]["step"])
        setattr(st, {"policy_optimizer_state_dict": "opt_pi", "q1_optimizer_state_dict": "opt_q1",
                     "q2_optimizer_state_dict": "opt_q2"}[name], ad)
    if hp.auto_entropy_tuning:
        st.log_alpha = float(np.asarray(ckpt["log_alpha"], np.float64))
        st.alpha = math.exp(st.log_alpha)
        ao = ckpt["alpha_optimizer_state_dict"]["state"].get(0)
        if ao is not None:
            st.opt_alpha_m = float(np.asarray(ao["exp_avg"], np.float64))
            st.opt_alpha_v = float(np.asarray(ao["exp_avg_sq"], np.float64))
            st.opt_alpha_step = float(ao["step"])
        st.alpha_orphaned = True
    else:
        st.alpha = float(F32(hp.alpha))
    return st
