"""Experiment logger (API of reference sac/utils/experiment_logger.py:16-148).

TensorBoard is optional: without ``torch.utils.tensorboard`` the scalars are
kept in memory (and the .npy dumps still work)."""
from __future__ import annotations

from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Optional


class _NullWriter:
    def __init__(self, *a, **k):
        self.scalars = []

    def add_scalar(self, tag, value, step=None):
        self.scalars.append((tag, float(value), step))

    def add_hparams(self, *a, **k):
        pass

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


def _flatten(d: Dict[str, Any], prefix: str = "") -> Dict[str, Any]:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "."))
        elif isinstance(v, (int, float, str, bool)) or v is None:
            out[key] = "None" if v is None else v
        else:
            out[key] = str(v)
    return out


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

    def log_q_values(self, q1: float, q2: float, step: int) -> None:
        self.metrics_writer.add_scalar("QValues/Q1", q1, step)
        self.metrics_writer.add_scalar("QValues/Q2", q2, step)
        self.q1_values.append(q1)
        self.q2_values.append(q2)

    def log_scalar(self, tag: str, value: float, step: int) -> None:
        self.metrics_writer.add_scalar(tag, value, step)

    def log_hparams(self, config: Dict[str, Any], metrics: Dict[str, float]) -> None:
        if self._hparams_logged:
            return
        hp = _flatten(config)
        mt = {f"hparam/{k}": float(v) for k, v in metrics.items()}
        self.hparams_writer.add_hparams(hp, mt)
        self._hparams_logged = True

    def close(self) -> None:
        self.metrics_writer.close()
        self.hparams_writer.close()
