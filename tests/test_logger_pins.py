"""SURVEY f4 pinned to the reference: the ExperimentLogger's writer calls.

tests/golden/make_golden.py recorded, through a stand-in SummaryWriter, every
call the reference's ExperimentLogger (sac/utils/experiment_logger.py:54-148)
makes for a fixed call sequence -- episode metrics, Q values, log_hparams with
the full SAC config and with no metrics, the log_q_values / log_episode_stats
gates, flush / close -- and for run_training_loop (agent.py:329-418) on DetEnv
(tests/golden/ref_logger.json, data only).  The same sequence through this
repo's logger must make the same calls: same writers (file suffixes), tags,
values, steps, flattened hparams ('/'-joined keys, str() of non-scalars) and
metrics ('placeholder_metric' when empty).  The loop part needs the engine:
tests/test_gpu_rollout.py::test_training_loop_logger_matches_reference."""
import json
import os

import numpy as np
import pytest

from _fixtures import GOLDEN

REF = json.load(open(os.path.join(GOLDEN, "ref_logger.json")))
LOGGER_CFG = {"enabled": True, "env_name": "Det", "agent_name": "SAC", "run_name": "pin", "use_timestamp": False,
              "timestamp_format": "%Y", "flush_secs": 10, "log_episode_stats": True, "log_q_values": True,
              "save_model": {"enabled": False, "path": None}}


def recording_writer(rec):
    class Writer:
        def __init__(self, log_dir=None, flush_secs=None, filename_suffix=""):
            self.suffix = filename_suffix

        def add_scalar(self, tag, value, step=None):
            rec.append(["add_scalar", self.suffix, tag, float(value), step])

        def add_hparams(self, hparam_dict, metric_dict, *a, **k):
            rec.append(["add_hparams", self.suffix, dict(hparam_dict), dict(metric_dict)])

        def flush(self):
            rec.append(["flush", self.suffix])

        def close(self):
            rec.append(["close", self.suffix])

    return Writer


def _norm(rec, tmp):
    return json.loads(json.dumps(rec).replace(str(tmp), "<log_dir>"))


def _full_cfg(tmp):
    """make_golden._cfg of the logger capture's config (c = obs 3, act 2, [16, 16], B 8, auto)."""
    return {
        "sac": {"gamma": 0.99, "tau": 0.005, "alpha": 0.1, "auto_entropy_tuning": True, "actor_lr": 3e-4,
                "critic_lr": 3e-4, "alpha_lr": 3e-4},
        "q_net": {"hidden_sizes": [16, 16], "hidden_layers_act": "relu", "output_activation": "identity"},
        "policy_net": {"hidden_sizes": [16, 16], "hidden_layers_act": "relu", "output_activation": "identity",
                       "log_std_min": -20, "log_std_max": 2, "action_scale": 1.0},
        "buffer": {"capacity": 1000},
        "train": {"gradient_steps_per_update": 1, "seed": 0, "batch_size": 8, "warming_steps": 10, "device": "cpu"},
        "logger": dict(LOGGER_CFG, log_dir=str(tmp)),
    }


@pytest.mark.parametrize("case,over", [("all_on", {}),
                                       ("gates_off", {"log_q_values": False, "log_episode_stats": False})])
def test_logger_api_calls_match_reference(case, over, tmp_path, monkeypatch):
    from sac.utils import experiment_logger as xl

    full = _full_cfg(tmp_path)
    rec = []
    monkeypatch.setattr(xl, "_writer_cls", lambda: recording_writer(rec))
    lg = xl.ExperimentLogger(dict(LOGGER_CFG, log_dir=str(tmp_path), **over))
    lg.log_episode_metrics(0, 1.5, 10)
    lg.log_episode_metrics(1, -2.25, 7)
    lg.log_q_values(0.25, -0.5, 3)
    lg.log_q_values(1.0, 2.0, 4)
    lg.log_hparams(full, {"total_episodes": 2, "best_avg_return": 1.5, "final_avg_return": -0.375})
    lg.log_hparams(full, {"ignored": 1.0})
    lg.flush()
    lg.close()
    rec.append(["lists", lg.episode_rewards, lg.episode_lengths, lg.q1_values, lg.q2_values])
    assert _norm(rec, tmp_path) == REF[f"api/{case}"]
    rec2 = []
    monkeypatch.setattr(xl, "_writer_cls", lambda: recording_writer(rec2))
    lg2 = xl.ExperimentLogger(dict(LOGGER_CFG, log_dir=str(tmp_path), **over))
    lg2.log_hparams({"a": {"b": [1, 2], "c": None, "d": True, "e": 2.5, "f": "x"}, "g": 3}, {})
    assert _norm(rec2, tmp_path) == REF[f"api/{case}/empty_metrics"]


def test_logger_context_manager_and_npy_dtypes(tmp_path, monkeypatch):
    from sac.utils import experiment_logger as xl
    from sac.utils.logger_utils import load_lengths, load_rewards, save_lengths, save_rewards

    rec = []
    monkeypatch.setattr(xl, "_writer_cls", lambda: recording_writer(rec))
    with xl.ExperimentLogger(dict(LOGGER_CFG, log_dir=str(tmp_path))) as lg:
        lg.log_episode_metrics(0, 1.0, 3)
    assert rec[-4:] == [["flush", "_metrics"], ["flush", "_hparams"], ["close", "_metrics"], ["close", "_hparams"]]
    save_rewards(lg.run_dir / "x", [1.5, -2.0])
    save_lengths(lg.run_dir / "x", [3, 4])
    d = REF["npy_dtypes"]  # what the reference's run_training_loop wrote
    assert str(np.load(lg.run_dir / "x" / "episode_rewards.npy").dtype) == d["rewards"]
    assert str(np.load(lg.run_dir / "x" / "episode_lengths.npy").dtype) == d["lengths"]
    assert load_rewards(lg.run_dir / "x") == [1.5, -2.0] and load_lengths(lg.run_dir / "x") == [3, 4]


def test_q_value_log_equals_eager_values_on_cpu(monkeypatch):
    """sac.agent.QValueLog (the loops' sync-free QValues/* path) logs, for every
    env step in order, exactly the reference's q.mean().item() values of that
    moment's critics, across flushes and a ring wrap (CPU agent: the eager
    torch forward on the module parameters)."""
    import torch

    from _gpu import FakeEnv
    from sac.agent import SAC, QValueLog

    cfg = _full_cfg("/tmp/unused")
    cfg["logger"]["enabled"] = False
    agent = SAC(FakeEnv(3, 2), cfg)
    got = []

    class L:
        def log_q_values(self, q1, q2, step):
            got.append((q1, q2, step))

    ql = QValueLog(agent, L(), every=4)
    g = np.random.default_rng(0)
    want = []
    step = 0
    for it in range(7):
        n = int(g.integers(1, 4))
        s = g.standard_normal((n, 3)).astype(np.float32)
        a = g.uniform(-1, 1, (n, 2)).astype(np.float32)
        with torch.no_grad():
            for i in range(n):
                st, ac = torch.from_numpy(s[i:i + 1]), torch.from_numpy(a[i:i + 1])
                want.append((agent.q_net1(st, ac).mean().item(), agent.q_net2(st, ac).mean().item(), step + 1 + i))
        ql.record(s, a, step + 1)
        step += n
        with torch.no_grad():  # the critics move between env steps (an update ran)
            for p in agent.q_net1.parameters():
                p.add_(0.01)
    ql.finish()
    # steps exact; values equal to BLAS rounding (a batched row's dot product
    # may round differently from the single-row one) ...
    assert [g_[2] for g_ in got] == [w[2] for w in want]
    np.testing.assert_allclose(np.array([g_[:2] for g_ in got]), np.array([w[:2] for w in want]), rtol=1e-6, atol=1e-7)
    # ... and bit-equal for one row per record, the single-env loop's case
    got.clear()
    ql1 = QValueLog(agent, L(), every=3)
    want1 = []
    for k in range(1, 8):
        s = g.standard_normal((1, 3)).astype(np.float32)
        a = g.uniform(-1, 1, (1, 2)).astype(np.float32)
        with torch.no_grad():
            st, ac = torch.from_numpy(s), torch.from_numpy(a)
            want1.append((agent.q_net1(st, ac).mean().item(), agent.q_net2(st, ac).mean().item(), k))
        ql1.record(s[0], a[0], k)
    ql1.finish()
    assert got == want1
    # one record() larger than the ring (2 * every rows: a vector env with
    # num_envs > 2 * q_values_flush_every) grows it instead of failing
    got.clear()
    ql2 = QValueLog(agent, L(), every=1)
    s = g.standard_normal((5, 3)).astype(np.float32)
    a = g.uniform(-1, 1, (5, 2)).astype(np.float32)
    with torch.no_grad():
        st, ac = torch.from_numpy(s), torch.from_numpy(a)
        q1, q2 = agent.q_net1(st, ac).reshape(-1), agent.q_net2(st, ac).reshape(-1)
    ql2.record(s, a, 1)
    ql2.record(s[:2], a[:2], 6)
    ql2.finish()
    assert [x[2] for x in got] == [1, 2, 3, 4, 5, 6, 7]
    np.testing.assert_allclose(np.array([x[:2] for x in got[:5]]), torch.stack([q1, q2], 1).numpy(), rtol=1e-6)
