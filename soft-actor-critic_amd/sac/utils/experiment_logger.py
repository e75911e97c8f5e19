"""Experiment logger (API of reference sac/utils/experiment_logger.py:16-148).

Same run directory, writers, tags and hparams record as the reference:
``Episode/Reward`` / ``Episode/Length`` (gated by ``log_episode_stats``),
``QValues/Q1`` / ``QValues/Q2`` (gated by ``log_q_values``), and ONE
``add_hparams`` call whose config is flattened with ``/``-joined keys (ints,
floats and bools kept, everything else ``str()``-ed) and whose metrics are
the given names as floats, ``{"placeholder_metric": 0.0}`` when empty
(reference :104-112, :129-148).  Pinned against the reference's own calls by
tests/test_logger_pins.py (tests/golden/ref_logger.json).

TensorBoard is optional: without ``torch.utils.tensorboard`` the writers keep
every call in memory (``_NullWriter.calls``), and the .npy dumps still work.
The engine's extra scalars (``Loss/*``, ``Alpha``, ``Perf/*``; sac.agent.LossLog)
go through ``log_scalar``."""
from __future__ import annotations

from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Optional


class _NullWriter:
    """In-memory stand-in for SummaryWriter: records (method, args) in order."""

    def __init__(self, *a, **k):
        self.calls = []
        self.scalars = []

    def add_scalar(self, tag, value, step=None):
        self.calls.append(("add_scalar", tag, float(value), step))
        self.scalars.append((tag, float(value), step))

    def add_hparams(self, hparam_dict, metric_dict, *a, **k):
        self.calls.append(("add_hparams", dict(hparam_dict), dict(metric_dict)))

    def flush(self):
        pass

    def close(self):
        pass


def _writer_cls():
    try:
        from torch.utils.tensorboard import SummaryWriter  # noqa: F401

        return SummaryWriter
    except Exception:
        return _NullWriter


def prepare_hparams(hparams: Dict[str, Any]) -> Dict[str, Any]:
    """Flatten a nested config into ``a/b/c`` keys; keep int / float / bool
    values and ``str()`` the rest (None -> 'None', lists -> '[256, 256]')."""
    flat: Dict[str, Any] = {}
    stack = [("", hparams)]
    while stack:
        prefix, value = stack.pop(0)
        if isinstance(value, dict):
            stack[0:0] = [(f"{prefix}/{k}" if prefix else k, v) for k, v in value.items()]
        else:
            flat[prefix] = value
    return {k: v if isinstance(v, (int, float, bool)) else str(v) for k, v in flat.items()}


class ExperimentLogger:
    def __init__(self, cfg: Dict[str, Any], run_name: Optional[str] = None, env_name: Optional[str] = None,
                 agent_name: Optional[str] = None):
        self.cfg = cfg
        self.env_name = env_name or cfg.get("env_name") or "Environment"
        self.agent_name = agent_name or cfg.get("agent_name") or "Agent"
        base = run_name or cfg.get("run_name") or "sac"
        if cfg.get("use_timestamp"):
            base = f"{base}-{datetime.now().strftime(cfg['timestamp_format'])}"
        self.run_id = base
        self.run_dir = Path(cfg["log_dir"]) / self.env_name / self.agent_name / self.run_id
        self.run_dir.mkdir(parents=True, exist_ok=True)
        W = _writer_cls()
        flush = cfg.get("flush_secs", 10)
        self.metrics_writer = W(self.run_dir.as_posix(), flush_secs=flush, filename_suffix="_metrics")
        self.hparams_writer = W(self.run_dir.as_posix(), flush_secs=flush, filename_suffix="_hparams")
        self._hparams_logged = False
        self.episode_rewards = []
        self.episode_lengths = []
        self.q1_values = []
        self.q2_values = []

    def log_episode_metrics(self, episode_idx: int, reward: float, length: int) -> None:
        if not self.cfg.get("log_episode_stats", True):
            return
        self.metrics_writer.add_scalar("Episode/Reward", reward, episode_idx)
        self.metrics_writer.add_scalar("Episode/Length", length, episode_idx)
        self.episode_rewards.append(reward)
        self.episode_lengths.append(length)

    def log_q_values(self, q1_value: float, q2_value: float, step: int) -> None:
        if not self.cfg.get("log_q_values", False):
            return
        self.metrics_writer.add_scalar("QValues/Q1", q1_value, step)
        self.metrics_writer.add_scalar("QValues/Q2", q2_value, step)
        self.q1_values.append(q1_value)
        self.q2_values.append(q2_value)

    def log_scalar(self, tag: str, value: float, step: int) -> None:
        """Engine scalars (Loss/*, Alpha, Perf/*): not in the reference, which logs no losses."""
        self.metrics_writer.add_scalar(tag, value, step)

    def log_hparams(self, hparams: Dict[str, Any], metrics: Dict[str, float]) -> None:
        if self._hparams_logged:
            return
        prepared_metrics = {k: float(v) for k, v in metrics.items()}
        if not prepared_metrics:
            prepared_metrics = {"placeholder_metric": 0.0}
        self.hparams_writer.add_hparams(prepare_hparams(hparams), prepared_metrics)
        self._hparams_logged = True

    def save_matplotlib_graphs(self) -> None:
        """Reward / length / Q-value curves as PDFs in the run directory."""
        from .logger_utils import make_and_save_graph

        tag = f"{self.env_name} - {self.agent_name}"
        stem = f"{self.env_name}_{self.agent_name}"
        if self.episode_rewards:
            make_and_save_graph(1, [self.episode_rewards], f"Episode Rewards Over Time - {tag}", "Episode", "Reward",
                                f"episode_rewards-{stem}.pdf", self.run_dir)
        if self.episode_lengths:
            make_and_save_graph(1, [self.episode_lengths], f"Episode Lengths Over Time - {tag}", "Episode", "Length",
                                f"episode_lengths-{stem}.pdf", self.run_dir)
        if self.q1_values and self.q2_values:
            make_and_save_graph(2, [self.q1_values, self.q2_values], f"Q-Values Over Time - {tag}", "Step",
                                "Q-Value", f"q_values-{stem}.pdf", self.run_dir, legend=["Q1", "Q2"])

    def flush(self) -> None:
        self.metrics_writer.flush()
        self.hparams_writer.flush()

    def close(self) -> None:
        self.flush()
        self.metrics_writer.close()
        self.hparams_writer.close()

    def __enter__(self) -> "ExperimentLogger":
        return self

    def __exit__(self, exc_type, exc_val, exc_tb) -> None:
        self.close()
