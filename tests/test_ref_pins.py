"""SURVEY f1-f3 pinned to the reference itself (CPU part).

tests/golden/make_golden.py ran the reference in the build container and
committed:
  ref_ckpt_c1_auto.pth  the file the reference's save_agent wrote after 2
                        injected steps (agent.py:521-536);
  ref_ckpt_c1_auto.npz  the reference continuing from there (cont/) and a fresh
                        reference agent after load_agent of that file (load/),
                        steps 3 and 4 with full post-step state;
  ref_loop.npz          run_training_loop (agent.py:329-418) on the
                        deterministic DetEnv: every training_step call as
                        (transitions pushed so far, len(replay_buffer)), and
                        the final deque rows.
Here: the checkpoint format, the oracle's load_agent restatement against both
continuations, and the batched driver's update count (sac.agent
.due_updates_gated) against the reference loop's calls for 1..7 envs."""
import os

import numpy as np
import pytest
import torch

from _fixtures import GOLDEN
from oracle import sac_oracle as O

CKPT = os.path.join(GOLDEN, "ref_ckpt_c1_auto.pth")
NETS = ("policy", "q1", "q2", "q1t", "q2t")
REF_KEYS = {"policy_net_state_dict", "q_net1_state_dict", "q_net2_state_dict", "q_net1_target_state_dict",
            "q_net2_target_state_dict", "policy_optimizer_state_dict", "q1_optimizer_state_dict",
            "q2_optimizer_state_dict", "log_alpha", "alpha_optimizer_state_dict"}


def _fx():
    import json

    fx = np.load(os.path.join(GOLDEN, "ref_ckpt_c1_auto.npz"))
    return fx, json.loads(str(fx["config"]))


def _np_ckpt():
    ck = torch.load(CKPT, map_location="cpu", weights_only=True)

    def conv(x):
        if isinstance(x, torch.Tensor):
            return x.detach().numpy()
        if isinstance(x, dict):
            return {k: conv(v) for k, v in x.items()}
        if isinstance(x, list):
            return [conv(v) for v in x]
        return x

    return conv(ck)


def test_reference_checkpoint_format():
    """The reference's own file loads with weights_only=True and holds the
    save_agent dict (auto-tuning: log_alpha + alpha optimizer)."""
    ck = torch.load(CKPT, map_location="cpu", weights_only=True)
    assert set(ck) == REF_KEYS
    assert ck["log_alpha"].dtype == torch.float64 and ck["log_alpha"].dim() == 0
    assert list(ck["policy_net_state_dict"]) == ["net.0.weight", "net.0.bias", "net.2.weight", "net.2.bias",
                                                 "net.4.weight", "net.4.bias"]
    st = ck["q1_optimizer_state_dict"]["state"]
    assert sorted(st) == list(range(6)) and float(st[0]["step"]) == 2.0
    assert ck["q1_optimizer_state_dict"]["param_groups"][0]["betas"] == (0.9, 0.999)


def _check(fx, st, prefix, k, losses):
    for got, want in zip(losses, fx[f"{prefix}/step{k}/out/losses"]):
        assert abs(got - want) <= 1e-4 * max(abs(want), 1e-2), (prefix, k, got, want)
    nets = {"policy": st.pi, "q1": st.q1, "q2": st.q2, "q1t": st.q1t, "q2t": st.q2t}
    for net in NETS:
        for key, val in nets[net].state_dict().items():
            full = f"{prefix}/step{k}/post/{net}/{key}"
            np.testing.assert_allclose(val, fx[full], rtol=0, atol=2e-6, err_msg=full)
    assert abs(st.log_alpha - float(fx[f"{prefix}/step{k}/post/log_alpha"])) < 1e-9


@pytest.mark.parametrize("prefix", ["cont", "load"])
def test_oracle_load_agent_matches_reference(prefix):
    """cont/: the saved state continued (the checkpoint carries the complete
    learner state); load/: the reference's load_agent on a fresh agent, whose
    alpha optimizer no longer owns log_alpha, so alpha stays as loaded while
    L_alpha is still computed (agent.py:550-554)."""
    fx, meta = _fx()
    hp = O.SacHyper.from_config(meta["cfg"])
    st = O.load_checkpoint(_np_ckpt(), hp, meta["act"])
    assert st.alpha_orphaned
    if prefix == "cont":
        st.alpha_orphaned = False
    for k in (3, 4):
        b = O.Batch(*(fx[f"step{k}/in/{x}"] for x in ("s", "a", "r", "s2", "d")))
        out = O.training_step(st, hp, b, fx[f"step{k}/in/eps_t"], fx[f"step{k}/in/eps_a"])
        _check(fx, st, prefix, k, out["losses"])
    if prefix == "load":
        assert st.log_alpha == float(fx["step2/post/log_alpha"])  # frozen at the loaded value


def test_checkpoint_holds_step2_state():
    fx, meta = _fx()
    ck = _np_ckpt()
    for net, key in (("policy", "policy_net_state_dict"), ("q1", "q_net1_state_dict"), ("q2t", "q_net2_target_state_dict")):
        for k, v in ck[key].items():
            assert np.array_equal(v, fx[f"step2/post/{net}/{k}"]), (net, k)


LOOP = np.load(os.path.join(GOLDEN, "ref_loop.npz"))
LOOP_TAGS = sorted({k.split("/")[0] for k in LOOP.files})


@pytest.mark.parametrize("tag", LOOP_TAGS)
@pytest.mark.parametrize("n_envs", [1, 2, 3, 4, 7])
def test_batched_update_count_matches_reference_loop(tag, n_envs):
    """run_vectorized_training_loop counts gradient steps per vector step with
    due_updates_gated (sac/agent.py); after every vector step of N envs the
    running total must equal the reference loop's training_step calls made by
    that many env steps, also across the warm-up boundary, with eviction
    (capacity 32) and when warming_steps > capacity (never updates)."""
    from sac.agent import due_updates_gated

    W, u, g, cap, _ = (int(x) for x in LOOP[f"{tag}/config"])
    calls = LOOP[f"{tag}/calls"]
    T = int(LOOP[f"{tag}/total_steps"])
    total = count = 0
    while total + n_envs <= T:
        len_before = min(cap, total)
        old, total = total, total + n_envs
        due = due_updates_gated(old, total, len_before, cap, W, u, g)
        if min(cap, total) >= W:  # SAC.can_update() after the push
            count += due
        want = int(np.sum(calls[:, 0] <= total))
        assert count == want, (tag, n_envs, total, count, want)
    # every call saw a buffer of at least warming_steps rows (agent.py:159-164)
    assert np.all(calls[:, 1] >= W)


def test_det_env_rows_are_policy_independent():
    """The deque rows of the reference loop are reproduced by stepping DetEnv
    with arbitrary actions (what makes them comparable across policies)."""
    import sys

    sys.path.insert(0, GOLDEN)
    from det_env import DetEnv

    tag = "w20_u2_g3_cap32"
    W, u, g, cap, n_ep = (int(x) for x in LOOP[f"{tag}/config"])
    env = DetEnv(3, 2)
    env.reset(seed=0)  # SAC._set_seed
    rows = []
    for _ in range(n_ep):
        s, _ = env.reset()
        done = False
        while not done:
            s2, r, te, tr, _ = env.step(np.ones(2, np.float32) * 7)
            done = te or tr
            rows.append((s, r, s2, done))
            s = s2
    rows = rows[-cap:]
    assert np.array_equal(np.stack([r[0] for r in rows]), LOOP[f"{tag}/mem_state"])
    assert np.array_equal(np.array([r[1] for r in rows]), LOOP[f"{tag}/mem_reward"])
    assert np.array_equal(np.stack([r[2] for r in rows]), LOOP[f"{tag}/mem_next_state"])
    assert np.array_equal(np.array([r[3] for r in rows]), LOOP[f"{tag}/mem_done"])
