"""SURVEY f1-f3 on the MI355X, pinned to the reference's own outputs
(tests/golden/ref_ckpt_c1_auto.{pth,npz}, ref_loop.npz; see test_ref_pins.py).

  * a checkpoint file written by the reference's save_agent loads into the
    engine (weights_only) and the next two injected steps match the reference
    after ITS load_agent (alpha frozen at the loaded value, agent.py:550-554)
    -- and, with train.alpha_after_load = "tune", the reference agent that
    simply continued;
  * the engine's save_agent writes the reference's dict, and the oracle's
    restatement of load_agent continues from it to the engine's next step;
  * run_training_loop and run_vectorized_training_loop (1 env) on DetEnv push
    the reference loop's rows and call the gradient step at the reference's
    env steps with the reference's buffer lengths.
Tolerances as tests/test_gpu_parity.py (fp32 parity mode)."""
import copy
import os
import sys

import numpy as np
import pytest
import torch

from _fixtures import GOLDEN
from oracle import sac_oracle as O

pytestmark = pytest.mark.gpu

CKPT = os.path.join(GOLDEN, "ref_ckpt_c1_auto.pth")
NETS = ("policy", "q1", "q2", "q1t", "q2t")


def _fx():
    import json

    fx = np.load(os.path.join(GOLDEN, "ref_ckpt_c1_auto.npz"))
    return fx, json.loads(str(fx["config"]))


def _agent(meta, seed=5, alpha_after_load=None):
    from _gpu import FakeEnv
    from sac.agent import SAC

    cfg = copy.deepcopy(meta["cfg"])
    cfg["train"].update(device="cuda", precision="fp32", seed=seed)
    if alpha_after_load:
        cfg["train"]["alpha_after_load"] = alpha_after_load
    cfg["buffer"]["capacity"] = 4 * cfg["train"]["batch_size"]
    return SAC(FakeEnv(meta["obs"], meta["act"]), cfg)


def _to_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, dict):
        return {k: _to_np(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_np(v) for v in x)
    return x


def _inject(agent, fx, k, B, A):
    b = [fx[f"step{k}/in/{x}"] for x in ("s", "a", "r", "s2", "d")]
    start = len(agent.replay_buffer)
    agent.replay_buffer.push_batch(*b)
    idx = torch.arange(start, start + B, dtype=torch.int32).reshape(1, B)
    e = torch.from_numpy(np.stack([fx[f"step{k}/in/eps_t"], fx[f"step{k}/in/eps_a"]])).reshape(1, 2, B, A)
    agent.engine.train(agent.replay_buffer, 1, indices=idx, eps=e)
    return agent.engine.losses()


def _nets(agent):
    return {"policy": agent.policy_net, "q1": agent.q_net1, "q2": agent.q_net2, "q1t": agent.q_net1_target,
            "q2t": agent.q_net2_target}


def _compare(agent, fx, prefix, k, losses, lr):
    for got, want in zip(losses, fx[f"{prefix}/step{k}/out/losses"]):
        assert abs(got - want) <= 1e-4 * max(abs(want), 1e-2), (prefix, k, got, want)
    for net, m in _nets(agent).items():
        for key, val in m.state_dict().items():
            d = np.abs(val.detach().cpu().numpy() - fx[f"{prefix}/step{k}/post/{net}/{key}"])
            assert d.max() <= 2 * lr * k + 1e-5, (prefix, k, net, key, d.max())
            assert np.mean(d <= 1e-6) >= 0.995, (prefix, k, net, key, np.mean(d <= 1e-6))


@pytest.mark.parametrize("mode,prefix", [(None, "load"), ("tune", "cont")])
def test_reference_checkpoint_loads_and_continues(mode, prefix):
    fx, meta = _fx()
    agent = _agent(meta, seed=5, alpha_after_load=mode)
    # the fresh agent's init differs from the checkpoint (seed 5 vs 0)
    assert not np.array_equal(agent.policy_net.state_dict()["net.0.weight"].cpu().numpy(),
                              fx["step2/post/policy/net.0.weight"])
    agent.load_agent(CKPT)
    la0 = float(agent.engine.alpha_state[0].item())
    assert la0 == float(fx["step2/post/log_alpha"])
    B, A = meta["batch"], meta["act"]
    for k in (3, 4):
        losses = _inject(agent, fx, k, B, A)
        _compare(agent, fx, prefix, k, losses, meta["cfg"]["sac"]["critic_lr"])
        la = float(agent.engine.alpha_state[0].item())
        want = float(fx[f"{prefix}/step{k}/post/log_alpha"])
        assert abs(la - want) <= 1e-7, (prefix, k, la, want)
    if prefix == "load":
        assert float(agent.engine.alpha_state[0].item()) == la0  # frozen, as the reference after load_agent
        assert float(agent.engine.opt_steps[3].item()) == 2.0   # the orphaned optimizer never steps


def test_engine_checkpoint_is_reference_format(tmp_path):
    """save_agent after a loaded + stepped engine: the reference's dict; the
    oracle's load_agent restatement continues from it to the engine's step."""
    fx, meta = _fx()
    agent = _agent(meta, alpha_after_load="tune")
    agent.load_agent(CKPT)
    B, A = meta["batch"], meta["act"]
    _inject(agent, fx, 3, B, A)
    path = str(tmp_path / "mine.pth")
    agent.save_agent(path)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    ref = torch.load(CKPT, map_location="cpu", weights_only=True)
    assert set(ck) == set(ref)
    for k in ref:
        if k.endswith("optimizer_state_dict"):
            assert sorted(ck[k]["state"]) == sorted(ref[k]["state"])
            assert float(ck[k]["state"][0]["step"]) == float(ref[k]["state"][0]["step"]) + 1
    conv = _to_np(ck)
    hp = O.SacHyper.from_config(meta["cfg"])
    st = O.load_checkpoint(conv, hp, A)
    st.alpha_orphaned = False  # "tune": the engine keeps tuning
    b = O.Batch(*(fx["step4/in/" + x] for x in ("s", "a", "r", "s2", "d")))
    want = O.training_step(st, hp, b, fx["step4/in/eps_t"], fx["step4/in/eps_a"])
    got = _inject(agent, fx, 4, B, A)
    for g, w in zip(got, want["losses"]):
        assert abs(g - w) <= 1e-4 * max(abs(w), 1e-2), (g, w)
    assert abs(float(agent.engine.alpha_state[0].item()) - st.log_alpha) <= 1e-7


# ---------------------------------------------------------------- loops (f1 / f2)
LOOP = np.load(os.path.join(GOLDEN, "ref_loop.npz"))
LOOP_TAGS = sorted({k.split("/")[0] for k in LOOP.files})


def _loop_cfg(W, u, g, cap):
    return {
        "sac": {"gamma": 0.99, "tau": 0.005, "alpha": 0.1, "auto_entropy_tuning": True, "actor_lr": 3e-4,
                "critic_lr": 3e-4, "alpha_lr": 3e-4},
        "q_net": {"hidden_sizes": [16, 16], "hidden_layers_act": "relu", "output_activation": "identity"},
        "policy_net": {"hidden_sizes": [16, 16], "hidden_layers_act": "relu", "output_activation": "identity",
                       "log_std_min": -20, "log_std_max": 2, "action_scale": 1.0},
        "buffer": {"capacity": cap},
        "train": {"gradient_steps_per_update": g, "update_frequency": u, "seed": 0, "batch_size": 8,
                  "warming_steps": W, "device": "cuda", "precision": "fp32"},
        "logger": {"enabled": False, "env_name": "DetEnv", "agent_name": "SAC", "log_episode_stats": False,
                   "log_q_values": False, "save_model": {"enabled": False, "path": None}},
    }


def _record(agent):
    pushed = [0]
    calls = []
    orig_store, orig_stores = agent.store_transition, agent.store_transitions

    def store(*a):
        pushed[0] += 1
        return orig_store(*a)

    def stores(states, *a):
        pushed[0] += len(states)
        return orig_stores(states, *a)

    agent.store_transition, agent.store_transitions = store, stores
    agent._run_updates = lambda n: calls.extend([(pushed[0], len(agent.replay_buffer))] * n)
    return calls


def _rows(agent):
    rb = agent.replay_buffer
    t = rb.gather(np.arange(len(rb)))
    return [x.cpu().numpy() for x in t]


@pytest.mark.parametrize("vectorized", [False, True])
@pytest.mark.parametrize("tag", LOOP_TAGS)
def test_training_loop_matches_reference_loop(tag, vectorized):
    sys.path.insert(0, GOLDEN)
    from det_env import DetEnv
    from sac.agent import SAC
    from sac.vector_env import SyncVectorEnv

    W, u, g, cap, n_ep = (int(x) for x in LOOP[f"{tag}/config"])
    T = int(LOOP[f"{tag}/total_steps"])
    env = SyncVectorEnv([lambda: DetEnv(3, 2)]) if vectorized else DetEnv(3, 2)
    agent = SAC(env, _loop_cfg(W, u, g, cap))
    calls = _record(agent)
    if vectorized:
        m = agent.run_vectorized_training_loop(T)
        assert m["total_env_steps"] == T
    else:
        m = agent.run_training_loop(n_ep, tqdm_disable=True)
    assert m["total_episodes"] == int(LOOP[f"{tag}/episodes"])
    assert m["final_avg_return"] == pytest.approx(float(LOOP[f"{tag}/final_avg_return"]), abs=1e-9)
    assert np.array_equal(np.array(calls, np.int64).reshape(-1, 2), LOOP[f"{tag}/calls"])
    s, _, r, s2, d = _rows(agent)
    assert np.array_equal(s, LOOP[f"{tag}/mem_state"])
    assert np.array_equal(r, LOOP[f"{tag}/mem_reward"].astype(np.float32))
    assert np.array_equal(s2, LOOP[f"{tag}/mem_next_state"])
    assert np.array_equal(d != 0, LOOP[f"{tag}/mem_done"])
