"""Run-artifact helpers (API of reference sac/utils/logger_utils.py:7-60).

``episode_rewards.npy`` is float32 and ``episode_lengths.npy`` int32, as the
reference writes them; the run directory is created if missing."""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Sequence

import numpy as np


def save_rewards(run_dir, rewards: Sequence[float]) -> None:
    run_dir = Path(run_dir)
    run_dir.mkdir(parents=True, exist_ok=True)
    np.save(run_dir / "episode_rewards.npy", np.array(rewards, dtype=np.float32))


def save_lengths(run_dir, lengths: Sequence[int]) -> None:
    run_dir = Path(run_dir)
    run_dir.mkdir(parents=True, exist_ok=True)
    np.save(run_dir / "episode_lengths.npy", np.array(lengths, dtype=np.int32))


def load_rewards(run_dir) -> List[float]:
    return np.load(Path(run_dir) / "episode_rewards.npy").astype(float).tolist()


def load_lengths(run_dir) -> List[int]:
    return np.load(Path(run_dir) / "episode_lengths.npy").astype(int).tolist()


def make_and_save_graph(number_of_curves: int, data: list, title: str, xlabel: str, ylabel: str, filename: str,
                        run_dir, legend: Optional[List[str]] = None) -> None:
    """``number_of_curves`` curves of ``data`` to ``run_dir/filename`` (needs
    matplotlib; a no-op without it).  The reference joins ``run_dir + "/" +
    filename``, which fails for the Path its logger passes; this joins paths."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # pragma: no cover - optional dependency
        return
    plt.figure()
    for i in range(number_of_curves):
        plt.plot(data[i])
    plt.title(title)
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    if legend:
        plt.legend(legend)
    plt.savefig(str(Path(run_dir) / filename))
    plt.close()
