"""Replay buffer resident in HBM (API of reference ``sac/replay_buffer.py``).

Storage is fp32 on the device, ring-ordered with ``(size, pos)`` mirrored on
the host and on the device, in one of two layouts (``layout=``):

* ``"records"`` (default): one ``[cap][row_stride]`` table of transition
  records ``obs | next_obs | act | rew | done | pad``, padded to whole 128-B
  lines (C2: 54 floats -> 64 = 256 B).  A sampled row is 2 cache lines; the
  replay-gather PMC profile measured 3.2x more bytes fetched than gathered for
  the struct-of-arrays form (scattered 4-B rew/done lines, 96-B obs rows
  straddling lines), DESIGN.md §2;
* ``"soa"``: struct-of-arrays ``obs[cap][O] | act[cap][A] | rew[cap] |
  next_obs[cap][O] | done[cap]``.

``obs``, ``act``, ``rew``, ``next_obs``, ``done`` are tensor views of the
fields in both layouts.

* ``push`` (replay_buffer.py:21-30) stages rows in pinned host memory; staged rows
  are appended by one HIP kernel (``torch.ops.sac_hip.replay_push``) before the next read, so an
  env loop pays one small H2D copy per flush, not per field.
* ``sample`` (replay_buffer.py:32-39) keeps the reference's RNG stream: indices
  come from Python ``random.sample`` over positions (oldest = 0, the deque order)
  so a seeded run selects exactly the rows the reference would; rows are gathered
  on the device (``torch.ops.sac_hip.replay_gather``) and returned as ``Transition``s.
* ``sample_tensors`` is the batched form used by ``SAC.sample_batch``: one
  Transition of device tensors.
* The fused engine path samples on the device itself (Feistel permutation keyed
  by Philox; distinct uniform rows like ``random.sample``), see DESIGN.md.
"""
from __future__ import annotations

import random
from collections import namedtuple
from typing import List, Optional

import numpy as np
import torch

from . import _engine as E
from ._engine import ops

Transition = namedtuple("Transition", ("state", "action", "reward", "next_state", "done"))


class ReplayBuffer:
    def __init__(self, capacity: int, device=None, obs_dim: Optional[int] = None,
                 act_dim: Optional[int] = None, stage_rows: int = 4096, layout: str = "records"):
        """Experience replay of at most ``capacity`` transitions (FIFO eviction)."""
        self.capacity = int(capacity)
        if self.capacity < 1:
            raise ValueError("capacity must be >= 1")
        if layout not in ("records", "soa"):
            raise ValueError("layout must be 'records' or 'soa'")
        self.layout = layout
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda" if torch.cuda.is_available() else "cpu")
        self._size = 0
        self._pos = 0
        self._stage_rows = int(stage_rows)
        self._staged: List[np.ndarray] = []
        self._n_staged = 0
        self.obs_dim = obs_dim
        self.act_dim = act_dim
        self._alloc_done = False
        if obs_dim is not None and act_dim is not None:
            self._alloc(obs_dim, act_dim)

    # ------------------------------------------------------------------ storage
    def _alloc(self, obs_dim: int, act_dim: int) -> None:
        E.require_gpu(self.device)
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        cap, dev = self.capacity, self.device
        O, A = self.obs_dim, self.act_dim
        f32 = dict(dtype=torch.float32, device=dev)
        self.row_width = 2 * O + A + 2
        if self.layout == "records":
            W = self.row_width
            self.row_stride = 16 if W <= 16 else (W + 31) // 32 * 32  # whole 64-B / 128-B lines
            self.records = torch.zeros(cap, self.row_stride, **f32)
            self.storage = self.records.view(-1)
            offs = [0, 2 * O, 2 * O + A, O, 2 * O + A + 1]  # obs, act, rew, next_obs, done
            self.obs = self.records[:, :O]
            self.next_obs = self.records[:, O:2 * O]
            self.act = self.records[:, 2 * O:2 * O + A]
            self.rew = self.records[:, 2 * O + A]
            self.done = self.records[:, 2 * O + A + 1]
        else:
            # one allocation, field-major: obs[cap][O] | act[cap][A] | rew[cap] | next_obs[cap][O] | done[cap]
            self.row_stride = 0
            self.storage = torch.zeros(cap * self.row_width, **f32)
            offs = [0, cap * O, cap * (O + A), cap * (O + A + 1), cap * (2 * O + A + 1)]
            self.obs = self.storage[offs[0]:offs[1]].view(cap, O)
            self.act = self.storage[offs[1]:offs[2]].view(cap, A)
            self.rew = self.storage[offs[2]:offs[3]]
            self.next_obs = self.storage[offs[3]:offs[4]].view(cap, O)
            self.done = self.storage[offs[4]:]
        self.state = torch.zeros(3, dtype=torch.int64, device=dev)  # size, next slot, push generation
        # the sac_hip custom ops' replay descriptor (csrc/sac_torch_ops.cpp)
        self.layout_spec = [cap, O, A, self.row_stride] + offs
        self._desc = E.ReplayDesc(
            self.obs.data_ptr(), self.act.data_ptr(), self.rew.data_ptr(), self.next_obs.data_ptr(),
            self.done.data_ptr(), cap, O, A, self.state.data_ptr(), self.row_stride)
        self._alloc_done = True

    @property
    def desc(self) -> E.ReplayDesc:
        self.flush()
        return self._desc

    def _row(self, state, action, reward, next_state, done) -> np.ndarray:
        s = np.asarray(state, dtype=np.float32).reshape(-1)
        a = np.asarray(action, dtype=np.float32).reshape(-1)
        s2 = np.asarray(next_state, dtype=np.float32).reshape(-1)
        if not self._alloc_done:
            self._alloc(s.size, a.size)
        row = np.empty(self.row_width, np.float32)
        O, A = self.obs_dim, self.act_dim
        row[:O] = s
        row[O:O + A] = a
        row[O + A] = np.float32(reward)
        row[O + A + 1:2 * O + A + 1] = s2
        row[-1] = np.float32(bool(done))
        return row

    # ------------------------------------------------------------------ reference API
    def push(self, state, action, reward, next_state, done) -> None:
        """Store a transition (replay_buffer.py:21-30)."""
        self._staged.append(self._row(state, action, reward, next_state, done))
        self._n_staged += 1
        if self._n_staged >= self._stage_rows:
            self.flush()

    def push_batch(self, states, actions, rewards, next_states, dones) -> None:
        """Append n transitions at once (device or host arrays; rows in order).

        Host inputs are packed into ONE pinned [n][2O+A+2] buffer: one H2D copy
        and one push kernel per batch (the vectorised rollout's per-step cost)."""
        if not any(isinstance(x, torch.Tensor) and x.is_cuda for x in (states, actions, rewards, next_states, dones)):
            st = np.asarray(states, np.float32)
            n = st.shape[0]
            if n == 0:
                return
            st = st.reshape(n, -1)
            ac = np.asarray(actions, np.float32).reshape(n, -1)
            if not self._alloc_done:
                self._alloc(st.shape[1], ac.shape[1])
            self.flush()
            O, A = self.obs_dim, self.act_dim
            host = torch.empty(n, self.row_width, dtype=torch.float32, pin_memory=torch.cuda.is_available())
            h = host.numpy()
            h[:, :O] = st
            h[:, O:O + A] = ac
            h[:, O + A] = np.asarray(rewards, np.float32).reshape(n)
            h[:, O + A + 1:2 * O + A + 1] = np.asarray(next_states, np.float32).reshape(n, -1)
            h[:, -1] = np.asarray(dones).reshape(n).astype(bool)
            self._push_device_rows(host.to(self.device, non_blocking=True))
            return
        st = torch.as_tensor(states, dtype=torch.float32)
        n = st.shape[0]
        if n == 0:
            return
        if not self._alloc_done:
            self._alloc(st.reshape(n, -1).shape[1], torch.as_tensor(actions).reshape(n, -1).shape[1])
        self.flush()
        dev = self.device
        rows = torch.cat([
            st.reshape(n, -1).to(dev),
            torch.as_tensor(actions, dtype=torch.float32).reshape(n, -1).to(dev),
            torch.as_tensor(rewards, dtype=torch.float32).reshape(n, 1).to(dev),
            torch.as_tensor(next_states, dtype=torch.float32).reshape(n, -1).to(dev),
            torch.as_tensor(dones).to(torch.float32).reshape(n, 1).to(dev),
        ], dim=1).contiguous()
        self._push_device_rows(rows)

    def _push_device_rows(self, rows: torch.Tensor) -> None:
        n = rows.shape[0]
        with torch.cuda.device(self.device):
            ops().replay_push(self.storage, self.state, self.layout_spec, rows, self._size, self._pos)
        self._size = min(self.capacity, self._size + n)
        self._pos = (self._pos + n) % self.capacity
        self._keep = rows  # keep alive until the kernel has consumed it

    def flush(self) -> None:
        """Append staged host rows with one H2D copy + one push kernel."""
        if not self._n_staged:
            return
        host = torch.from_numpy(np.stack(self._staged)).pin_memory() if torch.cuda.is_available() \
            else torch.from_numpy(np.stack(self._staged))
        rows = host.to(self.device, non_blocking=True)
        self._staged.clear()
        self._n_staged = 0
        self._push_device_rows(rows)
        self._keep_host = host

    def __len__(self) -> int:
        return min(self.capacity, self._size + self._n_staged)

    def _check(self, batch_size: int) -> None:
        if len(self) < batch_size:
            raise ValueError(
                f"Not enough samples in the replay buffer to sample {batch_size} transitions. "
                f"Current size: {len(self)}")

    def sample_indices(self, batch_size: int) -> List[int]:
        """Logical positions (0 = oldest), drawn exactly like ``random.sample``
        over the reference deque (same consumption of Python's ``random``)."""
        self._check(batch_size)
        return random.sample(range(len(self)), batch_size)

    def gather(self, logical_idx) -> Transition:
        """Device gather of the given logical positions -> Transition of tensors."""
        self.flush()
        idx = torch.as_tensor(logical_idx, dtype=torch.int32).reshape(-1)
        idx = idx.to(self.device, non_blocking=True)
        with torch.cuda.device(self.device):
            return Transition(*ops().replay_gather(self.storage, self.state, self.layout_spec, idx))

    def sample_gather_device(self, batch_size: int, seed: int, step: int):
        """Device sampler + gather in one kernel: (indices, Transition) of
        ``batch_size`` distinct rows for RNG (seed, step)."""
        self._check(batch_size)
        self.flush()
        with torch.cuda.device(self.device):
            idx, *t = ops().replay_sample_gather(self.storage, self.state, self.layout_spec, batch_size, seed, step)
        return idx, Transition(*t)

    def sample_tensors(self, batch_size: int) -> Transition:
        return self.gather(self.sample_indices(batch_size))

    def sample(self, batch_size: int) -> List[Transition]:
        """List of ``batch_size`` distinct transitions (replay_buffer.py:32-39).

        Each field is a host numpy row (float32); ``done`` is a bool, ``reward`` a
        Python float, as pushed."""
        t = self.sample_tensors(batch_size)
        s, a, r, s2, d = (x.cpu().numpy() for x in t)
        return [Transition(s[i], a[i], float(r[i]), s2[i], bool(d[i] != 0)) for i in range(batch_size)]

    def clear(self) -> None:
        self._size = self._pos = 0
        self._staged.clear()
        self._n_staged = 0
        if self._alloc_done:
            # size and write slot back to 0; the push generation moves on, so a
            # batch the engine staged before the clear is never used after it
            self.state[:2].zero_()
            self.state[2:].add_(1)

