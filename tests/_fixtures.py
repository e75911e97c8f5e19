"""Helpers shared by the tests: load golden fixtures, build oracle states."""
import json
import os

import numpy as np

from oracle import sac_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONFIGS = ["c1_fixed", "c1_auto", "elu3_clamp", "mix_act", "gelu_tanh", "const_reward", "c2", "donkey_new"]
FULL_INIT = ["c1_fixed", "c1_auto", "elu3_clamp", "mix_act", "gelu_tanh", "const_reward"]


def load(name):
    fx = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    meta = json.loads(str(fx["config"]))
    return fx, meta


def summary(t):
    f = np.asarray(t, np.float64).ravel()
    idx = np.linspace(0, f.size - 1, num=min(64, f.size)).astype(np.int64)
    s = np.zeros(64)
    s[: idx.size] = f[idx]
    return np.concatenate([[f.sum(), (f * f).sum()], s])


def batch(fx, k):
    return O.Batch(*(fx[f"step{k}/in/{x}"] for x in ("s", "a", "r", "s2", "d")))


def eps(fx, k):
    return fx[f"step{k}/in/eps_t"], fx[f"step{k}/in/eps_a"]


def init_state_dicts(name):
    """Initial weights of the 5 nets for a fixture: from the fixture when it holds
    them in full, else re-created with the reference seeding via sac.models."""
    fx, meta = load(name)
    cfg = meta["cfg"]
    out = {}
    if name in FULL_INIT:
        for net in ("policy", "q1", "q2", "q1t", "q2t"):
            out[net] = {k.split("/", 2)[2]: fx[k] for k in fx.files if k.startswith(f"init/{net}/") and "#" not in k}
        return out
    from sac.models import PolicyNetwork, QNetwork

    seed = cfg["train"]["seed"]
    pc, qc = cfg["policy_net"], cfg["q_net"]
    pi = PolicyNetwork(meta["obs"], meta["act"], pc["hidden_sizes"], seed=seed,
                       hidden_activations=pc["hidden_layers_act"])
    q1 = QNetwork(meta["obs"], meta["act"], qc["hidden_sizes"], qc["hidden_layers_act"], seed=seed)
    q2 = QNetwork(meta["obs"], meta["act"], qc["hidden_sizes"], qc["hidden_layers_act"], seed=seed + 1)
    for net, m in (("policy", pi), ("q1", q1), ("q2", q2), ("q1t", q1), ("q2t", q2)):
        out[net] = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    return out


def oracle_state(name):
    fx, meta = load(name)
    cfg = meta["cfg"]
    hp = O.SacHyper.from_config(cfg)
    sds = init_state_dicts(name)
    qa, pa = cfg["q_net"]["hidden_layers_act"], cfg["policy_net"]["hidden_layers_act"]
    pi = O.MLP.from_state_dict(sds["policy"], pa)
    q1 = O.MLP.from_state_dict(sds["q1"], qa)
    q2 = O.MLP.from_state_dict(sds["q2"], qa)
    st = O.SacState.fresh(pi, q1, q2, hp, meta["act"])
    st.q1t = O.MLP.from_state_dict(sds["q1t"], qa)
    st.q2t = O.MLP.from_state_dict(sds["q2t"], qa)
    return st, hp, fx, meta
