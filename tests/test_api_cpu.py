"""Host-side API mirror without a GPU: construction follows the reference
(sac/agent.py:22-124, sac/models.py, sac/replay_buffer.py), the hot path fails
loudly instead of falling back to a CPU implementation, and the bench's
algorithmic FLOP count equals SURVEY §8(d)."""
import copy

import numpy as np
import pytest
import torch

from _fixtures import load
from _gpu import FakeEnv


def _cfg(name="c1_auto"):
    _, meta = load(name)
    cfg = copy.deepcopy(meta["cfg"])
    cfg["train"]["device"] = "cpu"
    cfg["logger"]["enabled"] = False
    return cfg, meta


def test_agent_constructs_reference_networks_on_cpu():
    from sac.agent import SAC

    cfg, meta = _cfg()
    agent = SAC(FakeEnv(meta["obs"], meta["act"]), cfg)
    assert agent.engine is None
    fx, _ = load("c1_auto")
    for net, m in (("policy", agent.policy_net), ("q1", agent.q_net1), ("q2", agent.q_net2)):
        for k, v in m.state_dict().items():
            key = f"init/{net}/{k}"
            if key in fx.files:
                assert np.array_equal(v.numpy(), fx[key]), key
    # targets start as copies of the critics (agent.py:75-76)
    for a, b in ((agent.q_net1, agent.q_net1_target), (agent.q_net2, agent.q_net2_target)):
        for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
            assert ka == kb and torch.equal(va, vb)
    assert agent.target_entropy == -float(meta["act"])


def test_hot_path_fails_loudly_without_gpu():
    from sac import _engine as E
    from sac.agent import SAC

    cfg, meta = _cfg()
    agent = SAC(FakeEnv(meta["obs"], meta["act"]), cfg)
    with pytest.raises(E.EngineUnavailable):
        agent.training_step()
    with pytest.raises(E.EngineUnavailable):
        agent.train_steps(4)
    with pytest.raises(E.EngineUnavailable):
        agent.select_action(np.zeros(meta["obs"], np.float32))
    with pytest.raises(E.EngineUnavailable):
        agent.store_transition(np.zeros(meta["obs"]), np.zeros(meta["act"]), 0.0, np.zeros(meta["obs"]), False)


def test_cpu_device_resolution(monkeypatch):
    """``train.device: cpu`` (the reference's CPU configs) stays on the host
    only without a HIP device or with ``engine_device: cpu``; with a device
    visible it moves to the engine's GPU (the GPU side: test_gpu_rollout)."""
    from sac.agent import resolve_device

    assert resolve_device({"device": "cpu"}) == torch.device("cpu")  # no GPU in this container
    with pytest.raises(ValueError):
        resolve_device({"device": "cpu", "engine_device": "gpu"})
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    with pytest.warns(UserWarning, match="MI355X engine"):
        assert resolve_device({"device": "cpu"}) == torch.device("cuda", 0)
    assert resolve_device({"device": "cpu", "engine_device": "cpu"}) == torch.device("cpu")
    assert resolve_device({"device": "cuda:0"}) == torch.device("cuda", 0)


def test_substeps_need_the_engine():
    """The reference sub-steps run on the engine's device state: without a GPU
    they fail loudly like the fused step (no CPU fallback)."""
    import torch

    from sac import _engine as E
    from sac.agent import SAC

    cfg, meta = _cfg()
    agent = SAC(FakeEnv(meta["obs"], meta["act"]), cfg)
    s = torch.zeros(4, meta["obs"])
    a = torch.zeros(4, meta["act"])
    r = torch.zeros(4)
    calls = {"compute_target_q_values": (r, r, s), "update_q_networks": (s, a, r), "update_policy_network": (s,),
             "update_entropy_temperature": (r,), "soft_update_target_networks": ()}
    for name, args in calls.items():
        with pytest.raises(E.EngineUnavailable):
            getattr(agent, name)(*args)


def test_replay_buffer_cpu_contract():
    from sac import _engine as E
    from sac.replay_buffer import ReplayBuffer, Transition

    assert Transition._fields == ("state", "action", "reward", "next_state", "done")
    with pytest.raises(ValueError):
        ReplayBuffer(0, device="cpu")
    rb = ReplayBuffer(10, device="cpu")
    assert len(rb) == 0
    with pytest.raises(ValueError, match="Not enough samples"):
        rb.sample(1)
    with pytest.raises(E.EngineUnavailable):
        ReplayBuffer(10, device="cpu", obs_dim=3, act_dim=1)


def test_models_api_and_errors():
    from sac.models import ACT_CODES, PolicyNetwork, QNetwork, build_mlp

    with pytest.raises(ValueError):
        build_mlp(4, [], 2)
    with pytest.raises(KeyError):  # unknown activation: KeyError, as the reference's dict lookup
        QNetwork(4, 1, [8], hidden_activations="swish")
    q = QNetwork(4, 1, [8, 8], seed=0)
    assert q(torch.zeros(3, 4), torch.zeros(3, 1)).shape == (3,)
    p = PolicyNetwork(4, 2, [8], seed=0, log_std_min=-5, log_std_max=1)
    mu, log_std = p(torch.zeros(3, 4) + 100.0)
    assert mu.shape == (3, 2) and float(log_std.max()) <= 1 and float(log_std.min()) >= -5
    assert set(ACT_CODES) >= {"relu", "tanh", "elu", "leaky_relu", "gelu", "selu", "identity"}


def test_bench_flops_match_survey():
    import bench

    want = {"c1": 9.06e6, "c2": 588.78e6, "c3": 9420.41e6, "c4": 597.69e6, "c4w": 911.21e6}
    for k, v in want.items():
        c = bench.CONFIGS[k]
        phases, total, _, _ = bench.gemm_flops(c["obs"], c["act"], c["hidden"], c["batch"])
        assert total == pytest.approx(v, rel=1e-4), k
        # per-phase counts (roofline of each kernel) add up to the step's F_alg
        assert sum(phases) == total


def test_due_updates_gated_matches_the_reference_per_step_loop():
    """The vectorised driver's gradient-step count for one vector step of N
    env steps equals the reference loop's (agent.py:355-369: push, then
    can_update() and t % update_frequency) counted env step by env step,
    including vector steps that cross the warm-up boundary, a full ring and
    warming_steps > capacity (never updates)."""
    import itertools

    from sac.agent import due_updates_gated

    for N, freq, grad, warm, cap in itertools.product((1, 3, 16), (1, 2, 5), (1, 3), (0, 7, 64, 100), (50, 1000)):
        length = total = 0
        for _ in range(40):
            want = 0
            ln = length
            for t in range(total + 1, total + N + 1):
                ln = min(cap, ln + 1)
                if warm <= cap and ln >= warm and t % freq == 0:
                    want += grad
            got = due_updates_gated(total, total + N, length, cap, warm, freq, grad)
            assert got == want, (N, freq, grad, warm, cap, total)
            length = min(cap, length + N)
            total += N
