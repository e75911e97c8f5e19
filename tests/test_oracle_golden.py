"""The CPU oracle against the golden vectors captured from the reference
(tests/golden/make_golden.py).  This pins the oracle before it is trusted as
the checker of the HIP engine."""
import numpy as np
import pytest

from _fixtures import CONFIGS, FULL_INIT, batch, eps, load, oracle_state, summary
from oracle import sac_oracle as O

NETS = ("policy", "q1", "q2", "q1t", "q2t")


def _net(st, name):
    return {"policy": st.pi, "q1": st.q1, "q2": st.q2, "q1t": st.q1t, "q2t": st.q2t}[name]


@pytest.mark.parametrize("name", CONFIGS)
def test_oracle_matches_reference(name):
    st, hp, fx, meta = oracle_state(name)
    for k in range(1, meta["steps"] + 1):
        et, ea = eps(fx, k)
        out = O.training_step(st, hp, batch(fx, k), et, ea)
        ref = fx[f"step{k}/out/losses"]
        for got, want in zip(out["losses"], ref):
            if np.isnan(want):
                assert np.isnan(got)
            else:
                assert abs(got - want) <= 1e-4 * max(abs(want), 1e-2), (k, got, want)
        np.testing.assert_allclose(out["y"], fx[f"step{k}/out/y"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(out["log_pi"], fx[f"step{k}/out/log_pi"], rtol=1e-5, atol=1e-5)
        for net in NETS:
            for key, val in _net(st, net).state_dict().items():
                full = f"step{k}/post/{net}/{key}"
                if full in fx.files:
                    np.testing.assert_allclose(val, fx[full], rtol=0, atol=2e-6, err_msg=full)
                else:
                    s = summary(val)
                    r = fx[full + "#summary"]
                    np.testing.assert_allclose(s[2:], r[2:], rtol=0, atol=2e-6, err_msg=full)
                    np.testing.assert_allclose(s[0], r[0], rtol=1e-5, atol=1e-3, err_msg=full)
        if st.log_alpha is not None:
            assert abs(st.log_alpha - float(fx[f"step{k}/post/log_alpha"])) < 1e-9


@pytest.mark.parametrize("name", FULL_INIT + ["c2", "donkey_new"])
def test_models_init_matches_reference(name):
    """sac.models with the reference seeding reproduces the reference init bit-exactly."""
    import json

    fx, _ = load(name)
    from sac.models import PolicyNetwork, QNetwork

    meta = json.loads(str(fx["config"]))
    cfg = meta["cfg"]
    seed = cfg["train"]["seed"]
    pc, qc = cfg["policy_net"], cfg["q_net"]
    pi = PolicyNetwork(meta["obs"], meta["act"], pc["hidden_sizes"], seed=seed,
                       hidden_activations=pc["hidden_layers_act"])
    q1 = QNetwork(meta["obs"], meta["act"], qc["hidden_sizes"], qc["hidden_layers_act"], seed=seed)
    q2 = QNetwork(meta["obs"], meta["act"], qc["hidden_sizes"], qc["hidden_layers_act"], seed=seed + 1)
    for net, m in (("policy", pi), ("q1", q1), ("q2", q2)):
        for k, v in m.state_dict().items():
            key = f"init/{net}/{k}"
            v = v.numpy()
            if key in fx.files:
                assert np.array_equal(v, fx[key]), key
            else:
                assert np.array_equal(summary(v)[2:], fx[key + "#summary"][2:]), key


def test_constant_reward_closed_form():
    """ConstantRewardEnv: every transition terminal => y == r exactly."""
    st, hp, fx, meta = oracle_state("const_reward")
    et, ea = eps(fx, 1)
    out = O.training_step(st, hp, batch(fx, 1), et, ea)
    assert np.array_equal(out["y"], np.ones_like(out["y"]))
    assert np.array_equal(fx["step1/out/y"], np.ones_like(out["y"]))


def test_replay_sampling_semantics():
    """random.sample over the deque (replay_buffer.py:32-39): the oracle deque and
    sampling by position over range(len) pick the same rows as the reference did."""
    import random

    fx = np.load(f"{__import__('_fixtures').GOLDEN}/replay_sample.npz")
    for key in fx.files:
        cap, n, B, seed = (int(t[1:]) if t[0] in "nbs" else int(t[3:]) for t in key.split("_"))
        buf = O.ReplayDeque(cap)
        for i in range(n):
            buf.push(np.array([i], np.float32), np.zeros(1, np.float32), float(i), np.array([i + 1], np.float32), False)
        random.seed(seed)
        got = [t.reward for t in buf.sample(B)]
        assert np.array_equal(np.array(got), fx[key])
        # position-based sampling (what sac.replay_buffer does) == deque sampling
        random.seed(seed)
        pos = random.sample(range(len(buf)), B)
        oldest = max(0, n - cap)
        assert np.array_equal(np.array([oldest + p for p in pos], np.float64), fx[key])


def test_replay_not_enough_raises():
    buf = O.ReplayDeque(10)
    with pytest.raises(ValueError):
        buf.sample(1)
