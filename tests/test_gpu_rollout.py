"""Vectorised rollout + batched training-loop driver on the MI355X (SURVEY §8
f1/f2).  The parity anchor is the reference loop itself (agent.py:329-418, as
mirrored by SAC.run_training_loop): with one env the batched driver must
produce the same replay rows and the same engine state bit for bit; with N envs
the batched action kernel and the single-copy push must equal their per-row
forms."""
import copy
import os
import sys

import numpy as np
import pytest
import torch

from _fixtures import GOLDEN

pytestmark = pytest.mark.gpu


def _cfg(batch=16, warming=24, update_frequency=1, grad_steps=1, precision="fp32", capacity=4096):
    return {
        "sac": {"gamma": 0.99, "tau": 0.005, "alpha": 0.2, "auto_entropy_tuning": True, "actor_lr": 3e-4,
                "critic_lr": 3e-4, "alpha_lr": 3e-4},
        "q_net": {"hidden_sizes": [32, 32], "hidden_layers_act": "relu", "output_activation": "identity"},
        "policy_net": {"hidden_sizes": [32, 32], "hidden_layers_act": "relu", "output_activation": "identity",
                       "log_std_min": -20, "log_std_max": 2, "action_scale": 1.0},
        "buffer": {"capacity": capacity},
        "train": {"gradient_steps_per_update": grad_steps, "update_frequency": update_frequency, "seed": 3,
                  "batch_size": batch, "warming_steps": warming, "device": "cuda", "precision": precision,
                  "graph_chunk": 4},
        "logger": {"enabled": False, "env_name": "probe", "agent_name": "SAC", "log_episode_stats": False,
                   "log_q_values": False, "save_model": {"enabled": False, "path": None}},
    }


def _env():
    from sac.envs import OneDPointMassReachEnv

    return OneDPointMassReachEnv(max_steps=9, action_low=-0.5, action_high=0.5, goal_tolerance=0.1)


def _replay_rows(agent):
    rb = agent.replay_buffer
    rb.flush()
    n = len(rb)
    torch.cuda.synchronize()
    return {k: getattr(rb, k)[:n].cpu().clone() for k in ("obs", "act", "rew", "next_obs", "done")}


@pytest.mark.parametrize("update_frequency,grad_steps", [(1, 1), (3, 5)])
def test_vectorized_loop_one_env_equals_reference_loop(update_frequency, grad_steps):
    from sac.agent import SAC
    from sac.vector_env import SyncVectorEnv

    cfg = _cfg(update_frequency=update_frequency, grad_steps=grad_steps)
    ref = SAC(_env(), copy.deepcopy(cfg))
    m_ref = ref.run_training_loop(num_episodes=12, tqdm_disable=True)
    T = len(ref.replay_buffer)
    assert ref.engine.steps_done > 0
    vec = SAC(SyncVectorEnv([_env]), copy.deepcopy(cfg))
    m_vec = vec.run_vectorized_training_loop(T)
    torch.cuda.synchronize()
    assert m_vec["total_env_steps"] == T and m_vec["total_episodes"] == m_ref["total_episodes"]
    assert m_vec["gradient_steps"] == ref.engine.steps_done == vec.engine.steps_done
    assert m_vec["final_avg_return"] == pytest.approx(m_ref["final_avg_return"], rel=0, abs=1e-9)
    ra, rb = _replay_rows(ref), _replay_rows(vec)
    for k in ra:
        assert torch.equal(ra[k], rb[k]), k
    sa, sb = ref.engine.state_tensors(), vec.engine.state_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_batched_actions_equal_per_row_actions():
    from sac.agent import SAC
    from sac.vector_env import SyncVectorEnv

    cfg = _cfg()
    agent = SAC(SyncVectorEnv([_env] * 37), cfg)
    obs = np.random.default_rng(0).standard_normal((37, 1)).astype(np.float32)
    batched = agent.select_actions(obs, deterministic=True)
    rows = np.stack([agent.select_action(obs[i], deterministic=True) for i in range(37)])
    assert batched.shape == (37, 1) and np.array_equal(batched, rows)
    # stochastic: N draws of one (N, A) noise block == the kernel on the same eps
    torch.manual_seed(9)
    a1 = agent.select_actions(obs)
    torch.manual_seed(9)
    eps = torch.distributions.utils._standard_normal((37, 1), torch.float32, agent.device)
    a2 = agent.engine.policy_act(torch.from_numpy(obs).cuda(), eps).cpu().numpy()
    assert np.array_equal(a1, a2)


@pytest.mark.parametrize("n", [1, 5, 300])
def test_batched_push_equals_per_row_push(n):
    from sac.replay_buffer import ReplayBuffer

    g = np.random.default_rng(n)
    s, s2 = g.standard_normal((n, 24)).astype(np.float32), g.standard_normal((n, 24)).astype(np.float32)
    a = g.uniform(-1, 1, (n, 4)).astype(np.float32)
    r = g.standard_normal(n)  # float64 rewards, as gym returns them
    d = g.random(n) < 0.3
    cap = 257  # wraps for n = 300
    rb1 = ReplayBuffer(cap, device="cuda", obs_dim=24, act_dim=4)
    rb2 = ReplayBuffer(cap, device="cuda", obs_dim=24, act_dim=4)
    rb1.push_batch(s, a, r, s2, d)
    for i in range(n):
        rb2.push(s[i], a[i], float(r[i]), s2[i], bool(d[i]))
    rb2.flush()
    torch.cuda.synchronize()
    assert len(rb1) == len(rb2) == min(n, cap)
    for k in ("obs", "act", "rew", "next_obs", "done", "state"):
        assert torch.equal(getattr(rb1, k), getattr(rb2, k)), k


def test_vectorized_loop_many_envs_runs_and_counts():
    from sac.agent import SAC
    from sac.vector_env import SyncVectorEnv

    cfg = _cfg(batch=32, warming=64, update_frequency=2, grad_steps=3, precision="bf16")
    agent = SAC(SyncVectorEnv([_env] * 16), cfg)
    m = agent.run_vectorized_training_loop(16 * 20)
    torch.cuda.synchronize()
    assert m["total_env_steps"] == 320 and len(agent.replay_buffer) == 320
    # the reference loop (agent.py:355-369) at env step t: push, then 3 gradient
    # steps if len(buffer) >= 64 and t % 2 == 0 -- counted per env step, also
    # inside the vector step that crosses the warm-up boundary (t = 49..64)
    want = sum(3 for t in range(1, 321) if t >= 64 and t % 2 == 0)
    assert want == 387
    assert m["gradient_steps"] == want
    assert agent.engine.steps_done == m["gradient_steps"]
    agent.engine.check()
    assert all(np.isfinite(agent.engine.losses()[:3]))


def test_loss_and_throughput_scalars_are_logged(tmp_path):
    """the training loops log Loss/Q1, Loss/Q2, Loss/Policy,
    Loss/Alpha, Alpha and Perf/* scalars every logger.log_losses_every gradient
    steps from async snapshots (no per-step host sync); the snapshot values are
    the engine's own losses."""
    from sac.agent import SAC
    from sac.utils.experiment_logger import ExperimentLogger
    from sac.vector_env import SyncVectorEnv

    cfg = _cfg(batch=16, warming=32, precision="fp32")
    cfg["logger"].update(enabled=False, log_dir=str(tmp_path), run_name="t", use_timestamp=False,
                         log_losses_every=8)
    agent = SAC(SyncVectorEnv([_env] * 4), cfg)
    logger = ExperimentLogger(cfg["logger"], env_name="probe", agent_name="SAC")
    m = agent.run_vectorized_training_loop(4 * 40, logger=logger)
    torch.cuda.synchronize()
    rec = {}
    for tag, v, step in logger.metrics_writer.scalars:
        rec.setdefault(tag, []).append((step, v))
    for tag in ("Loss/Q1", "Loss/Q2", "Loss/Policy", "Loss/Alpha", "Alpha", "Perf/GradientStepsPerSec",
                "Perf/EnvStepsPerSec"):
        assert tag in rec and len(rec[tag]) >= 2, (tag, rec.keys())
        assert all(np.isfinite(v) for _, v in rec[tag]), tag
        steps = [s for s, _ in rec[tag]]
        assert steps == sorted(steps) and steps[-1] <= m["gradient_steps"]
    assert all(v > 0 for _, v in rec["Perf/GradientStepsPerSec"])
    # a snapshot is exactly the engine's stats at that step: re-snapshot now and compare
    from sac.agent import LossLog

    ll = LossLog(agent.engine, logger, 1)
    ll.after_updates(m["total_env_steps"])
    ll.finish()
    l = agent.engine.losses()
    last = {tag: rec2[-1][1] for tag, rec2 in _group(logger.metrics_writer.scalars).items()}
    assert last["Loss/Q1"] == pytest.approx(l[0], rel=1e-6) and last["Loss/Policy"] == pytest.approx(l[2], rel=1e-6)
    assert last["Alpha"] == pytest.approx(float(agent.engine.alpha_state[1]), rel=1e-12)


def _group(scalars):
    out = {}
    for tag, v, step in scalars:
        out.setdefault(tag, []).append((step, v))
    return out


def _rec_writer(rec):
    from test_logger_pins import recording_writer

    return recording_writer(rec)


def test_training_loop_logger_matches_reference(tmp_path, monkeypatch):
    """SURVEY f4/f2 against the reference's own run_training_loop record
    (tests/golden/ref_logger.json 'loop': DetEnv, logger on, log_q_values on,
    4 episodes): the same writer calls per tag -- QValues/Q1, QValues/Q2 at
    every env step (values from this run's critics: the reference's came from
    its random policy), Episode/Reward and Episode/Length per episode with the
    reference's values, and one add_hparams of the flattened config and the
    returned metrics (train/device 'cuda' here) -- while the Q values come
    through QValueLog with no .item() inside the loop."""
    import json

    import torch

    from sac import agent as agent_mod
    from sac.agent import SAC
    from sac.utils import experiment_logger as xl
    from test_logger_pins import LOGGER_CFG

    sys.path.insert(0, GOLDEN)
    from det_env import DetEnv

    ref = json.load(open(os.path.join(GOLDEN, "ref_logger.json")))
    cfg = json.loads(json.dumps(ref["loop_config"]).replace("<log_dir>", str(tmp_path)))
    cfg["train"]["device"] = "cuda"
    rec = []
    monkeypatch.setattr(xl, "_writer_cls", lambda: _rec_writer(rec))
    agent = SAC(DetEnv(3, 2), cfg)
    # eager per-step values at record time (the reference's q.mean().item()), for comparison
    eager = []
    orig_record = agent_mod.QValueLog.record

    def spy(self, states, actions, first_step):
        with torch.no_grad():
            s = torch.as_tensor(np.asarray(states, np.float32)).reshape(1, -1).to(agent.device)
            a = torch.as_tensor(np.asarray(actions, np.float32)).reshape(1, -1).to(agent.device)
            eager.append((first_step, self.agent.q_net1(s, a).mean(), self.agent.q_net2(s, a).mean()))
        return orig_record(self, states, actions, first_step)

    monkeypatch.setattr(agent_mod.QValueLog, "record", spy)
    items = []
    orig_item = torch.Tensor.item
    monkeypatch.setattr(torch.Tensor, "item", lambda t: items.append(1) or orig_item(t))
    m = agent.run_training_loop(4, tqdm_disable=True)
    n_items = len(items)
    monkeypatch.setattr(torch.Tensor, "item", orig_item)
    assert n_items == 0, "a .item() host sync ran inside the training loop"
    assert agent.engine.steps_done > 0  # updates ran (warming_steps 10)
    assert {k: float(v) for k, v in m.items()} == ref["loop_metrics"]
    norm = json.loads(json.dumps(rec).replace(str(tmp_path), "<log_dir>"))
    want = ref["loop"]

    def by_tag(calls):
        out = {}
        for c in calls:
            key = c[2] if c[0] == "add_scalar" else c[0]
            out.setdefault(key, []).append(c)
        return out

    got_t, want_t = by_tag(norm), by_tag(want)
    assert sorted(got_t) == sorted(want_t)
    for tag in ("Episode/Reward", "Episode/Length"):
        assert got_t[tag] == want_t[tag], tag
    for tag in ("QValues/Q1", "QValues/Q2"):
        assert [c[4] for c in got_t[tag]] == [c[4] for c in want_t[tag]], tag  # steps
    (gh,), (wh,) = got_t["add_hparams"], want_t["add_hparams"]
    assert gh[2].pop("train/device") == "cuda" and wh[2].pop("train/device") == "cpu"
    assert gh == wh
    # the async values are the per-step eager ones
    e = {st: (q1.item(), q2.item()) for st, q1, q2 in eager}
    for c1, c2 in zip(got_t["QValues/Q1"], got_t["QValues/Q2"]):
        assert (c1[3], c2[3]) == e[c1[4]]


def test_cpu_device_config_trains_on_the_engine():
    """A reference config with ``train.device: cpu`` (hparam_search/configs/
    inverted_pendulum.yaml:38) drops in: the agent moves to the HIP device,
    builds the engine, and runs the reference loop bit-identically to the same
    config written with ``device: cuda``."""
    from sac.agent import SAC

    cfg = _cfg()
    cpu_cfg = copy.deepcopy(cfg)
    cpu_cfg["train"]["device"] = "cpu"
    with pytest.warns(UserWarning, match="runs on the MI355X engine"):
        a = SAC(_env(), cpu_cfg)
    assert a.device.type == "cuda" and a.engine is not None
    assert a.config["train"]["device"] == "cpu"  # the logged hparam stays as written
    # one agent at a time: construction seeds the process-wide RNGs the loop draws from
    a.run_training_loop(num_episodes=6, tqdm_disable=True)
    b = SAC(_env(), copy.deepcopy(cfg))
    b.run_training_loop(num_episodes=6, tqdm_disable=True)
    torch.cuda.synchronize()
    assert a.engine.steps_done == b.engine.steps_done > 0
    sa, sb = a.engine.state_tensors(), b.engine.state_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
