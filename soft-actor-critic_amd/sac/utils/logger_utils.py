"""Run-artifact helpers (reference sac/utils/logger_utils.py:7-60)."""
from __future__ import annotations

from pathlib import Path
from typing import Sequence

import numpy as np


def save_rewards(run_dir, rewards: Sequence[float]) -> Path:
    path = Path(run_dir) / "episode_rewards.npy"
    np.save(path, np.asarray(rewards, dtype=np.float64))
    return path


def save_lengths(run_dir, lengths: Sequence[int]) -> Path:
    path = Path(run_dir) / "episode_lengths.npy"
    np.save(path, np.asarray(lengths, dtype=np.int64))
    return path


def make_and_save_graph(values: Sequence[float], title: str, ylabel: str, path) -> None:
    """Plot a curve to ``path`` when matplotlib is available (no-op otherwise)."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover - optional dependency
        return
    fig, ax = plt.subplots()
    ax.plot(np.asarray(values))
    ax.set_title(title)
    ax.set_xlabel("Episode")
    ax.set_ylabel(ylabel)
    fig.savefig(path)
    plt.close(fig)
