"""Host wrapper of one SAC learner on the HIP engine.

``SacEngine`` owns the device state the fused kernels read and write:

* one flat fp32 buffer per network (pi, Q1, Q2, Q1-target, Q2-target); every
  ``nn.Parameter`` of the modules is re-pointed to a view of it, so
  ``state_dict()`` / ``load_state_dict`` stay authoritative and checkpoints keep
  the reference's format (sac/agent.py:521-554);
* flat Adam ``exp_avg`` / ``exp_avg_sq`` buffers, exposed per parameter inside
  real ``torch.optim.Adam`` objects (state_dict-compatible);
* ``alpha_state`` = [log_alpha, alpha, m, v] in float64 (agent.py:43-55);
* optimizer step counters, the device RNG step and a stats block
  (losses[4], y[B], log_pi[B]) that is read only on demand (no per-step sync);
* the engine workspace (packed MFMA copies of the weights, activations).
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import _engine as E
from .models import ACT_CODES

PRECISIONS = {"fp32": E.PREC_FP32, "bf16": E.PREC_BF16}


def _flatten_into(module: nn.Module, flat: torch.Tensor) -> None:
    """Copy the module's Linear params into ``flat`` (layer order W, b) and make
    each parameter a view of it."""
    off = 0
    for lin in [m for m in module.modules() if isinstance(m, nn.Linear)]:
        for p in (lin.weight, lin.bias):
            n = p.numel()
            flat[off:off + n].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + n].view_as(p)
            off += n
    assert off == flat.numel()


def _param_count(module: nn.Module) -> int:
    return sum(p.numel() for m in module.modules() if isinstance(m, nn.Linear) for p in (m.weight, m.bias))


def _views(flat: torch.Tensor, like: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    out, off = [], 0
    for p in like:
        n = p.numel()
        out.append(flat[off:off + n].view_as(p))
        off += n
    return out


class SacEngine:
    def __init__(self, policy_net, q_net1, q_net2, q_net1_target, q_net2_target, *, batch_size: int,
                 gamma: float, tau: float, actor_lr: float, critic_lr: float, alpha_lr: float,
                 alpha: float, auto_entropy_tuning: bool, device, precision: str = "fp32",
                 seed: int = 0, betas=(0.9, 0.999), eps: float = 1e-8, layout: Optional[dict] = None):
        """``layout`` (tests and A/B runs only; None = the engine's choice, which
        every measured number uses): kernel layout overrides, the fields of
        sac_engine_config named in sac._engine.LAYOUT_KEYS -- layout ("auto" |
        "roles" | "rows" | "pairs"; an override the shape cannot take fails in
        create), stage_path (1 force / -1 refuse the stage path),
        stage_batch (-1: phase A gathers its own batch), upd_parts (batch parts
        of the large-batch update tiles), upd_threads (512 / 1024)."""
        self.device = torch.device(device)
        E.require_gpu(self.device)
        self.lib = E.load_library()
        self.precision = precision
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self.batch = int(batch_size)
        self.nets = dict(pi=policy_net, q1=q_net1, q2=q_net2, q1t=q_net1_target, q2t=q_net2_target)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.flat: Dict[str, torch.Tensor] = {}
        for k, net in self.nets.items():
            self.flat[k] = torch.zeros(_param_count(net), **f32)
            _flatten_into(net, self.flat[k])
        self.m = {k: torch.zeros_like(self.flat[k]) for k in ("pi", "q1", "q2")}
        self.v = {k: torch.zeros_like(self.flat[k]) for k in ("pi", "q1", "q2")}
        self.auto = bool(auto_entropy_tuning)
        self.alpha_state = torch.zeros(4, dtype=torch.float64, device=self.device)
        if self.auto:
            la = float(np.log(alpha))
            self.alpha_state[0] = la
            self.alpha_state[1] = math.exp(la)
        else:
            self.alpha_state[1] = float(np.float32(alpha))  # torch.tensor(alpha) is fp32 (agent.py:55)
        self.opt_steps = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.rng_step = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.stats = torch.full((4 + 2 * self.batch,), float("nan"), **f32)

        pi, q = policy_net, q_net1
        cfg = E.EngineConfig()
        cfg.obs_dim, cfg.act_dim, cfg.batch = pi.obs_size, pi.action_size, self.batch
        ql, qd = E.net_dims(q.linears())
        pl, pd = E.net_dims(pi.linears())
        if ql > E.MAX_LAYERS or pl > E.MAX_LAYERS:
            raise ValueError(f"at most {E.MAX_LAYERS - 1} hidden layers are supported")
        cfg.q_layers, cfg.pi_layers = ql, pl
        for i, d in enumerate(qd):
            cfg.q_dims[i] = d
        for i, d in enumerate(pd):
            cfg.pi_dims[i] = d
        cfg.q_hidden_act = ACT_CODES[q.hidden_activations]
        cfg.q_out_act = ACT_CODES[q.output_activation]
        cfg.pi_hidden_act = ACT_CODES[pi.hidden_activations]
        cfg.pi_out_act = ACT_CODES[pi.output_activation]
        cfg.gamma, cfg.tau = gamma, tau
        cfg.log_std_min, cfg.log_std_max, cfg.action_scale = pi.log_std_min, pi.log_std_max, pi.action_scale
        cfg.actor_lr, cfg.critic_lr, cfg.alpha_lr = actor_lr, critic_lr, alpha_lr
        cfg.beta1, cfg.beta2, cfg.adam_eps = betas[0], betas[1], eps
        cfg.auto_entropy = int(self.auto)
        cfg.target_entropy = -float(pi.action_size)
        cfg.precision = PRECISIONS[precision]
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        for k, v in (layout or {}).items():
            if k not in E.LAYOUT_KEYS:
                raise ValueError(f"unknown layout override {k!r} (one of {E.LAYOUT_KEYS})")
            setattr(cfg, k, E.LAYOUTS[v] if k == "layout" else int(v))
        self.cfg = cfg
        ws = self.lib.sac_engine_workspace_bytes(ctypes.byref(cfg))
        if ws == 0:
            E.check(-1)
        self.workspace = torch.empty(ws + 256, dtype=torch.uint8, device=self.device)
        base = (self.workspace.data_ptr() + 255) & ~255
        bufs = E.EngineBuffers(
            self.flat["pi"].data_ptr(), self.flat["q1"].data_ptr(), self.flat["q2"].data_ptr(),
            self.flat["q1t"].data_ptr(), self.flat["q2t"].data_ptr(),
            self.m["pi"].data_ptr(), self.v["pi"].data_ptr(), self.m["q1"].data_ptr(), self.v["q1"].data_ptr(),
            self.m["q2"].data_ptr(), self.v["q2"].data_ptr(), self.alpha_state.data_ptr(),
            self.opt_steps.data_ptr(), self.rng_step.data_ptr(), self.stats.data_ptr(), base, ws)
        self._bufs = bufs
        h = ctypes.c_void_p()
        E.check(self.lib.sac_engine_create(ctypes.byref(cfg), ctypes.byref(bufs), self._stream(), ctypes.byref(h)))
        self.handle = h
        self.ops = E.ops()
        # the caller-owned tensors the step reads and writes, sac_engine_buffers
        # order: the mutated arguments of torch.ops.sac_hip.train_step / train_graph
        self.state_list = [self.flat[k] for k in ("pi", "q1", "q2", "q1t", "q2t")] + [
            t for k in ("pi", "q1", "q2") for t in (self.m[k], self.v[k])] + [
            self.alpha_state, self.opt_steps, self.rng_step, self.stats, self.workspace]
        self.steps_done = 0
        # lazy hand-off status: an async D2H copy of the engine's status words
        # into pinned memory every STATUS_EVERY train calls, checked when it has
        # landed (never a per-step synchronisation); losses()/check() force it
        self._status = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        self._status_ev: Optional[torch.cuda.Event] = None
        self._calls = 0
        self.lib.sac_engine_uses_roles.argtypes = [ctypes.c_void_p]
        self.roles = bool(self.lib.sac_engine_uses_roles(h))
        # pair-tile kernels (csrc/sac_pairs.h): layout={"layout": "pairs"}
        self.lib.sac_engine_uses_pairs.argtypes = [ctypes.c_void_p]
        self.pairs = bool(self.lib.sac_engine_uses_pairs(h))
        # large-batch stage path (csrc/sac_wide.h): launches per step, 0 when the phase kernels run
        self.lib.sac_engine_uses_wide.argtypes = [ctypes.c_void_p]
        self.wide = int(self.lib.sac_engine_uses_wide(h))
        pl = (ctypes.c_int32 * 4)()
        self.lib.sac_engine_phase_launches.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.sac_engine_phase_launches(h, pl)
        self.phase_launches = list(pl)  # launches per step of phases A, B, C, D

    # ------------------------------------------------------------------ plumbing
    def _stream(self):
        return E.stream_handle(self.device)

    def close(self) -> None:
        if getattr(self, "handle", None):
            torch.cuda.synchronize(self.device)
            self.lib.sac_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    alpha_updates = True

    def set_alpha_update(self, enabled: bool) -> None:
        """Temperature (log alpha) Adam updates on/off (see sac_engine.h)."""
        E.check(self.lib.sac_engine_set_alpha_update(self.handle, int(bool(enabled)), self._stream()))
        self.alpha_updates = bool(enabled)

    def sync_params(self) -> None:
        """Re-pack the MFMA compute copies after host-side parameter changes."""
        E.check(self.lib.sac_engine_sync_params(self.handle, self._stream()))

    def param_views(self, key: str) -> List[torch.Tensor]:
        net = self.nets[key]
        return [p for m in net.modules() if isinstance(m, nn.Linear) for p in (m.weight, m.bias)]

    def adam_views(self, key: str):
        like = self.param_views(key)
        return _views(self.m[key], like), _views(self.v[key], like)

    def state_tensors(self) -> Dict[str, torch.Tensor]:
        """Every device tensor the step reads and writes (parameters, Adam
        moments, alpha state, step counters, RNG step)."""
        out = {f"param/{k}": v for k, v in self.flat.items()}
        out.update({f"m/{k}": v for k, v in self.m.items()})
        out.update({f"v/{k}": v for k, v in self.v.items()})
        out.update(alpha_state=self.alpha_state, opt_steps=self.opt_steps, rng_step=self.rng_step)
        return out

    def snapshot(self) -> Dict[str, torch.Tensor]:
        return {k: v.clone() for k, v in self.state_tensors().items()}

    def restore(self, snap: Dict[str, torch.Tensor]) -> None:
        """Copy a snapshot back in place and re-pack the compute copies."""
        for k, v in self.state_tensors().items():
            v.copy_(snap[k])
        self.sync_params()

    # ------------------------------------------------------------------ status
    STATUS_EVERY = 16

    def _raise_timeout(self) -> None:
        raise E.HandoffTimeout(
            "a workgroup hand-off of the SAC phase kernels timed out (the GPU was too contended for the "
            "role-split step to make progress): the gradient steps since the last good status are invalid")

    def _poll_status(self, block: bool = False) -> None:
        """Check the last status copy if it has landed (block: wait for a fresh one)."""
        if block:
            self._issue_status()
        ev = self._status_ev
        if ev is None:
            return
        if block:
            ev.synchronize()
        elif not ev.query():
            return
        self._status_ev = None
        if int(self._status[1]) != 0:
            self._raise_timeout()

    def _issue_status(self) -> None:
        E.check(self.lib.sac_engine_read_status(self.handle, ctypes.c_void_p(self._status.data_ptr()),
                                                self._stream()))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._status_ev = ev

    def _after_launch(self) -> None:
        self._calls += 1
        if self._status_ev is None and self._calls % self.STATUS_EVERY == 0:
            self._issue_status()

    def clear_status(self) -> None:
        """Reset the hand-off timeout flag (after handling a HandoffTimeout)."""
        self._status_ev = None
        E.check(self.lib.sac_engine_clear_status(self.handle, self._stream()))

    # ------------------------------------------------------------------ compute
    def train(self, replay, n_steps: int = 1, indices: Optional[torch.Tensor] = None,
              eps: Optional[torch.Tensor] = None) -> None:
        """n gradient steps.  indices: [n][B] int32 logical rows; eps: [n][2][B][A]."""
        if len(replay) < self.batch:
            replay._check(self.batch)
        replay.flush()
        if indices is not None:
            indices = indices.to(self.device, torch.int32).contiguous()
        if eps is not None:
            eps = eps.to(self.device, torch.float32).contiguous()
        self._poll_status()
        with torch.cuda.device(self.device):
            self.ops.train_step(self.handle.value, self.state_list, replay.storage, replay.state,
                                replay.layout_spec, int(n_steps), indices, eps)
        self._keep = (indices, eps)
        self.steps_done += n_steps
        self._after_launch()

    def train_graph(self, replay, n_steps: int, chunk: int = 32) -> None:
        if len(replay) < self.batch:
            replay._check(self.batch)
        replay.flush()
        self._poll_status()
        with torch.cuda.device(self.device):
            self.ops.train_graph(self.handle.value, self.state_list, replay.storage, replay.state,
                                 replay.layout_spec, int(n_steps), int(chunk))
        self.steps_done += n_steps
        if n_steps:
            self._after_launch()

    def policy_act(self, obs: torch.Tensor, eps: Optional[torch.Tensor] = None, want_log_pi: bool = False):
        obs = obs.to(self.device, torch.float32).contiguous()
        if eps is not None:
            eps = eps.to(self.device, torch.float32).contiguous()
        with torch.cuda.device(self.device):
            act, lp = self.ops.policy_act(self.handle.value, obs, eps, int(self.cfg.act_dim),
                                          bool(want_log_pi and eps is not None))
        return (act, lp if lp.numel() else None) if want_log_pi else act

    def time_phases(self, replay, n_steps: int) -> List[float]:
        """[A, B, C, D, gap]: mean hipEvent interval per phase launch (ms) and
        that of an empty kernel launched the same way (see sac_engine.h)."""
        out = (ctypes.c_float * 5)()
        E.check(self.lib.sac_engine_time_phases(self.handle, ctypes.byref(replay.desc), int(n_steps), out,
                                                self._stream()))
        self.steps_done += n_steps
        return list(out)

    # ------------------------------------------------------------------ readback (syncs)
    def check(self) -> None:
        """Raise HandoffTimeout if an in-launch hand-off of the phase kernels timed out."""
        self._poll_status(block=True)

    def losses(self) -> List[float]:
        """[L_Q1, L_Q2, L_pi, L_alpha] of the last step (NaN L_alpha when fixed).
        Raises HandoffTimeout if any step since the last check was invalid."""
        self._poll_status(block=True)
        return self.stats[:4].double().cpu().tolist()

    def last_targets(self) -> torch.Tensor:
        return self.stats[4:4 + self.batch]

    def last_log_pi(self) -> torch.Tensor:
        return self.stats[4 + self.batch:4 + 2 * self.batch]
