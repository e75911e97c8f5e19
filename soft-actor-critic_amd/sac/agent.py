"""Soft Actor-Critic agent (API of reference ``sac/agent.py``) on the MI355X engine.

``SAC(env, config)`` accepts the reference's YAML config unchanged and exposes
the same attributes and methods.  What changes is underneath:

* ``training_step`` (agent.py:302-327) is ONE call into ``libsac_engine.so``:
  four HIP kernels (sample+target+critic-backward, critic update, actor, actor
  update) on the current stream, no host synchronisation and no ``.item()``;
* the replay buffer lives in HBM (``sac.replay_buffer``);
* ``select_action`` (agent.py:149-156) runs the policy head in a HIP kernel.

Extra (optional) config keys, all under ``train``:
    precision: 'fp32' (default; exact-fp32 MFMA products, the reference's arithmetic) |
               'bf16' (opt-in: bf16 MFMA products, fp32 accumulate and master weights;
               loss deviation from the fp32 reference up to ~2e-3 rel)
    rng:       'device' (default; Philox/Feistel on the GPU, graph-replayable) |
               'reference' (Python ``random.sample`` indices + torch eps draws,
               the reference's RNG consumption)
    graph_chunk: steps per captured hipGraph for ``train_steps`` (default 32)
    engine_device: 'auto' (default) | 'cpu'.  The reference's ``device: cpu``
               configs (e.g. hparam_search/configs/inverted_pendulum.yaml:38)
               run unchanged: with 'auto' and a HIP device visible, the agent
               trains on the engine (``cuda:<current device>``) and warns once;
               'cpu' keeps the networks on the host, where the hot path raises
               ``EngineUnavailable`` (there is no CPU fallback).

After ``load_agent`` with auto-tuning, alpha stays frozen as in the reference
(it rebinds ``log_alpha`` but not its optimizer, agent.py:550-554); the
optional ``train.alpha_after_load: tune`` keeps tuning it instead.

Per-env-step ``QValues/*`` logging (``logger.log_q_values``) runs without the
reference's ``.item()`` syncs (``QValueLog``), in both training loops.
"""
from __future__ import annotations

import os
import pprint
import random
import time
import warnings
from collections import deque
from copy import deepcopy
from typing import Callable, Any, Dict, Optional

import numpy as np
import torch
import torch.optim as optim

from . import _engine as E
from .engine import SacEngine
from .models import PolicyNetwork, QNetwork
from .replay_buffer import ReplayBuffer, Transition

try:  # progress bars are optional
    from tqdm import tqdm as _tqdm
except Exception:  # pragma: no cover
    def _tqdm(it, disable=False):
        return it


def _make_logger(cfg, env_name, agent_name):
    from .utils.experiment_logger import ExperimentLogger

    return ExperimentLogger(cfg, env_name=env_name, agent_name=agent_name)


def resolve_device(train_cfg: dict) -> torch.device:
    """Device the agent trains on.  ``train.device`` as written, except that a
    reference config asking for ``cpu`` moves to the HIP device when one is
    visible (``train.engine_device: auto``, the default): the step only exists
    as the engine, and the reference's CPU configs should drop in unchanged."""
    dev = torch.device(train_cfg["device"])
    mode = train_cfg.get("engine_device", "auto")
    if mode not in ("auto", "cpu"):
        raise ValueError(f"train.engine_device must be 'auto' or 'cpu', got {mode!r}")
    if dev.type == "cpu" and mode == "auto" and torch.cuda.is_available():
        gpu = torch.device("cuda", torch.cuda.current_device())
        warnings.warn(f"train.device is 'cpu': the SAC step runs on the MI355X engine, training on {gpu} "
                      "(train.engine_device: cpu keeps the host device)", stacklevel=3)
        return gpu
    return dev


def due_updates(old_steps: int, new_steps: int, update_frequency: int, gradient_steps: int) -> int:
    """Gradient steps the reference loop runs while its env-step counter goes
    from old_steps to new_steps: ``gradient_steps`` at every step t with
    t % update_frequency == 0 (agent.py:361-364)."""
    return (new_steps // update_frequency - old_steps // update_frequency) * gradient_steps


def due_updates_gated(old_steps: int, new_steps: int, len_before: int, capacity: int, warming_steps: int,
                      update_frequency: int, gradient_steps: int) -> int:
    """``due_updates`` restricted to the env steps at which the reference's
    ``can_update()`` already holds (agent.py:159-164, 361-362): env step t
    (old_steps < t <= new_steps) pushes the (t - old_steps)-th of this vector
    step's transitions, after which the buffer holds min(capacity, len_before +
    t - old_steps) rows; it updates only if that is >= warming_steps."""
    if warming_steps > capacity or new_steps <= old_steps:
        return 0
    first = old_steps + max(1, warming_steps - len_before)  # first env step with can_update() true
    if first > new_steps:
        return 0
    return due_updates(first - 1, new_steps, update_frequency, gradient_steps)


class LossLog:
    """Loss and throughput scalars for the logger without per-step host syncs
    (the reference logs none: agent.py:324 drops the alpha
    dict and the losses are never read).  Every ``every`` gradient steps it
    queues an async device->pinned copy of the last step's [L_Q1, L_Q2, L_pi,
    L_alpha, alpha] behind the training launches and logs the previous
    snapshot once its event has completed; ``finish`` waits for the last one.
    Tags: Loss/Q1, Loss/Q2, Loss/Policy, Loss/Alpha (auto-tuning only), Alpha,
    Perf/GradientStepsPerSec, Perf/EnvStepsPerSec (host wall clock between
    snapshots), all at the gradient-step count of the snapshot."""

    TAGS = ("Loss/Q1", "Loss/Q2", "Loss/Policy", "Loss/Alpha", "Alpha")

    def __init__(self, engine: SacEngine, logger, every: int):
        self.engine, self.logger, self.every = engine, logger, max(1, int(every))
        self.buf = torch.zeros(5, dtype=torch.float64, pin_memory=torch.cuda.is_available())
        self.ev: Optional[torch.cuda.Event] = None
        self.pending_step = 0
        self.next_at = self.every
        self.t0 = time.perf_counter()
        self.grad0 = engine.steps_done
        self.env0 = 0

    def _emit(self) -> None:
        vals = self.buf.tolist()
        for tag, v in zip(self.TAGS, vals):
            if not (tag == "Loss/Alpha" and v != v):  # NaN L_alpha: fixed temperature
                self.logger.log_scalar(tag, v, self.pending_step)
        self.ev = None

    def after_updates(self, env_steps: int) -> None:
        eng = self.engine
        if eng.steps_done < self.next_at:
            return
        if self.ev is not None:
            if not self.ev.query():
                return  # the previous snapshot has not landed: skip this one, never block
            self._emit()
        now = time.perf_counter()
        dt = max(now - self.t0, 1e-9)
        self.logger.log_scalar("Perf/GradientStepsPerSec", (eng.steps_done - self.grad0) / dt, eng.steps_done)
        self.logger.log_scalar("Perf/EnvStepsPerSec", (env_steps - self.env0) / dt, eng.steps_done)
        self.t0, self.grad0, self.env0 = now, eng.steps_done, env_steps
        with torch.cuda.device(eng.device):
            snap = torch.cat([eng.stats[:4].double(), eng.alpha_state[1:2]])
            self.buf.copy_(snap, non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record()
        self.pending_step = eng.steps_done
        self.next_at = (eng.steps_done // self.every + 1) * self.every

    def finish(self) -> None:
        if self.ev is not None:
            self.ev.synchronize()
            self._emit()


class QValueLog:
    """``QValues/Q1`` and ``QValues/Q2`` per env step (agent.py:370-376,
    493-500) without the reference's two ``.item()`` host syncs per env step.

    ``record`` evaluates Q1 and Q2 of the env steps' (next state, action)
    pairs under the critics of that moment -- an eager forward on the
    engine-owned parameters, queued behind that env step's gradient steps --
    into a device buffer of [n][2]; the host inputs go up through pinned
    memory (non-blocking), so nothing waits.  Every ``every`` env steps (and
    at ``finish``) the filled rows are copied to pinned host memory behind the
    training launches, and ``logger.log_q_values(q1, q2, step)`` runs for each
    of them once that copy's event has completed (polled, never waited for,
    except by ``finish``).  Values are the reference's: the mean over a batch
    of one row is that row's value, as float32."""

    def __init__(self, agent: "SAC", logger, every: int = 256):
        self.agent, self.logger, self.every = agent, logger, max(1, int(every))
        self.cap = 2 * self.every
        self.dev = torch.empty(self.cap, 2, dtype=torch.float32, device=agent.device)
        self.fill = 0
        self.steps = []
        self.pending = []

    def record(self, states: Any, actions: Any, first_step: int) -> None:
        """Q of rows (states[i], actions[i]) logged at step first_step + i."""
        a = self.agent
        host = np.concatenate([np.asarray(states, np.float32).reshape(-1, a.obs_size),
                               np.asarray(actions, np.float32).reshape(-1, a.action_size)], axis=1)
        n = host.shape[0]
        if self.fill + n > self.cap:
            self._flush()
        if n > self.cap:  # one call larger than the ring (num_envs > 2 * every): grow it
            self.cap = n
            self.dev = torch.empty(self.cap, 2, dtype=torch.float32, device=a.device)
        x = torch.from_numpy(np.ascontiguousarray(host))
        if a.device.type == "cuda":
            x = x.pin_memory().to(a.device, non_blocking=True)
        s, act = x[:, :a.obs_size], x[:, a.obs_size:]
        with torch.no_grad():
            self.dev[self.fill:self.fill + n, 0] = a.q_net1(s, act).reshape(-1)
            self.dev[self.fill:self.fill + n, 1] = a.q_net2(s, act).reshape(-1)
        self.steps.extend(range(first_step, first_step + n))
        self.fill += n
        if self.fill >= self.every:
            self._flush()
        self._drain(block=False)

    def _flush(self) -> None:
        if not self.fill:
            return
        cuda = self.dev.is_cuda
        host = torch.empty(self.fill, 2, dtype=torch.float32, pin_memory=cuda)
        host.copy_(self.dev[:self.fill], non_blocking=cuda)
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record()
        # later record() writes to self.dev queue behind this copy on the stream
        self.pending.append((ev, host, self.steps))
        self.steps, self.fill = [], 0

    def _drain(self, block: bool) -> None:
        while self.pending:
            ev, host, steps = self.pending[0]
            if ev is not None:
                if not block and not ev.query():
                    return
                ev.synchronize()
            for (q1, q2), st in zip(host.tolist(), steps):
                self.logger.log_q_values(q1, q2, st)
            self.pending.pop(0)

    def finish(self) -> None:
        self._flush()
        self._drain(block=True)


class SAC:
    def __init__(self, env, config: dict):
        self.env = env
        self.config = config
        self.device = resolve_device(config["train"])
        self.replay_buffer = ReplayBuffer(config["buffer"]["capacity"], device=self.device)
        self.obs_size = env.observation_space.shape[0]
        self.action_size = env.action_space.shape[0]
        # same construction order (and therefore torch RNG use) as the reference
        self._init_policy_network()
        self._init_q_networks()
        self._init_optimizers()
        self._set_seed(config["train"]["seed"])

        self.target_entropy = -float(self.action_size)
        sac_cfg = config["sac"]
        self._auto = bool(sac_cfg["auto_entropy_tuning"])
        tr = config["train"]
        self.precision = tr.get("precision", "fp32")
        self.rng_mode = tr.get("rng", "device")
        self.graph_chunk = int(tr.get("graph_chunk", 32))
        self.engine: Optional[SacEngine] = None
        self._fixed_alpha = torch.tensor(sac_cfg["alpha"]).to(self.device)
        self.alpha_optimizer = None
        if self.device.type == "cuda":
            self._build_engine()

        self.env_name = config["logger"]["env_name"] or self._infer_env_name(env)
        self.agent_name = config["logger"]["agent_name"] or self.__class__.__name__
        self.logger = (_make_logger(config["logger"], self.env_name, self.agent_name)
                       if config["logger"]["enabled"] else None)

    # ------------------------------------------------------------------ construction
    def _init_q_networks(self) -> None:
        qc, seed = self.config["q_net"], self.config["train"]["seed"]
        kw = dict(obs_size=self.obs_size, action_size=self.action_size, hidden_sizes=qc["hidden_sizes"],
                  hidden_activations=qc["hidden_layers_act"], output_activation=qc["output_activation"])
        self.q_net1 = QNetwork(seed=seed, **kw).to(self.device)
        self.q_net2 = QNetwork(seed=seed + 1, **kw).to(self.device)
        self.q_net1_target = deepcopy(self.q_net1).to(self.device)
        self.q_net2_target = deepcopy(self.q_net2).to(self.device)

    def _init_policy_network(self) -> None:
        pc = self.config["policy_net"]
        self.policy_net = PolicyNetwork(
            obs_size=self.obs_size, action_size=self.action_size, hidden_sizes=pc["hidden_sizes"],
            log_std_min=pc["log_std_min"], log_std_max=pc["log_std_max"], action_scale=pc["action_scale"],
            hidden_activations=pc["hidden_layers_act"], output_activation=pc["output_activation"],
            seed=self.config["train"]["seed"]).to(self.device)

    def _init_optimizers(self) -> None:
        s = self.config["sac"]
        self.policy_optimizer = optim.Adam(self.policy_net.parameters(), lr=s["actor_lr"])
        self.q1_optimizer = optim.Adam(self.q_net1.parameters(), lr=s["critic_lr"])
        self.q2_optimizer = optim.Adam(self.q_net2.parameters(), lr=s["critic_lr"])

    def _set_seed(self, seed: int) -> None:
        np.random.seed(seed)
        torch.manual_seed(seed)
        random.seed(seed)
        self.env.reset(seed=seed)
        self.env.action_space.seed(seed)
        self.env.observation_space.seed(seed)

    def _build_engine(self) -> None:
        s, tr = self.config["sac"], self.config["train"]
        self.engine = SacEngine(
            self.policy_net, self.q_net1, self.q_net2, self.q_net1_target, self.q_net2_target,
            batch_size=tr["batch_size"], gamma=s["gamma"], tau=s["tau"], actor_lr=s["actor_lr"],
            critic_lr=s["critic_lr"], alpha_lr=s["alpha_lr"], alpha=s["alpha"],
            auto_entropy_tuning=self._auto, device=self.device, precision=self.precision,
            seed=int(tr.get("engine_seed", tr["seed"])))
        eng = self.engine
        # torch.optim.Adam objects whose state IS the engine's device state
        for opt, key in ((self.policy_optimizer, "pi"), (self.q1_optimizer, "q1"), (self.q2_optimizer, "q2")):
            ms, vs = eng.adam_views(key)
            for p, m, v in zip(eng.param_views(key), ms, vs):
                opt.state[p] = {"step": torch.tensor(0.0), "exp_avg": m, "exp_avg_sq": v}
        if self._auto:
            self.log_alpha = eng.alpha_state[0]
            self.alpha_optimizer = optim.Adam([self.log_alpha], lr=s["alpha_lr"])
            self.alpha_optimizer.state[self.log_alpha] = {
                "step": torch.tensor(0.0), "exp_avg": eng.alpha_state[2], "exp_avg_sq": eng.alpha_state[3]}

    def _engine(self) -> SacEngine:
        if self.engine is None:
            E.require_gpu(self.device)
        return self.engine

    @property
    def alpha(self) -> torch.Tensor:
        """Current temperature: float64 0-dim when auto-tuned (agent.py:50), fp32 otherwise."""
        if self._auto and self.engine is not None:
            return self.engine.alpha_state[1]
        return self._fixed_alpha

    # ------------------------------------------------------------------ data
    def store_transition(self, state: Any, action: Any, reward: float, next_state: Any, done: bool) -> None:
        self.replay_buffer.push(state, action, reward, next_state, done)

    def warmup_replay_buffer(self, env: Any, steps: int) -> None:
        state, _ = env.reset()
        for _ in range(steps):
            action = env.action_space.sample()
            next_state, reward, terminated, truncated, _ = env.step(action)
            done = terminated or truncated
            self.store_transition(state, action, reward, next_state, done)
            state = next_state
            if done:
                state, _ = env.reset()

    def select_action(self, state: Any, deterministic: bool = False) -> Any:
        """Policy action for one observation (HIP policy kernel; agent.py:149-156)."""
        eng = self._engine()
        obs = torch.as_tensor(np.asarray(state, dtype=np.float32)).reshape(1, -1).to(self.device)
        if deterministic:
            act = eng.policy_act(obs)
        else:
            eps = torch.distributions.utils._standard_normal((1, self.action_size), torch.float32, self.device)
            act = eng.policy_act(obs, eps)
        return act.cpu().numpy()[0]

    def select_actions(self, states: Any, deterministic: bool = False) -> np.ndarray:
        """Policy actions for N observations [N, obs]: one H2D copy, ONE policy
        kernel, one D2H copy (the batched form of ``select_action``; row i draws
        its noise from the same torch generator stream as N single calls would
        for N = 1)."""
        eng = self._engine()
        host = np.ascontiguousarray(np.asarray(states, dtype=np.float32).reshape(-1, self.obs_size))
        obs = torch.from_numpy(host)
        if self.device.type == "cuda":
            obs = obs.pin_memory().to(self.device, non_blocking=True)
        if deterministic:
            act = eng.policy_act(obs)
        else:
            eps = torch.distributions.utils._standard_normal((host.shape[0], self.action_size), torch.float32,
                                                             self.device)
            act = eng.policy_act(obs, eps)
        return act.cpu().numpy()

    def store_transitions(self, states: Any, actions: Any, rewards: Any, next_states: Any, dones: Any) -> None:
        """N transitions in env order: one pinned H2D copy + one push kernel."""
        self.replay_buffer.push_batch(states, actions, rewards, next_states, dones)

    def _run_updates(self, n: int) -> None:
        """n consecutive gradient steps (agent.py:361-364): one engine call, no
        host sync (device RNG); per-step calls in reference-RNG mode."""
        if n <= 0:
            return
        if self.rng_mode == "reference":
            for _ in range(n):
                self.training_step()
            return
        self.replay_buffer._check(self.config["train"]["batch_size"])
        if n >= self.graph_chunk:
            self._engine().train_graph(self.replay_buffer, n, self.graph_chunk)
        else:
            self._engine().train(self.replay_buffer, n)

    def can_update(self) -> bool:
        if self.config["train"]["warming_steps"] > self.config["buffer"]["capacity"]:
            print("Warning: warming_steps is greater than replay buffer capacity.")
        return len(self.replay_buffer) >= self.config["train"]["warming_steps"]

    def sample_batch(self) -> Transition:
        """Minibatch as device tensors (agent.py:166-193), reference RNG order."""
        return self.replay_buffer.sample_tensors(self.config["train"]["batch_size"])

    # ------------------------------------------------------------------ the hot path
    def _reference_rng_inputs(self):
        B, A = self.config["train"]["batch_size"], self.action_size
        idx = torch.tensor(self.replay_buffer.sample_indices(B), dtype=torch.int32)
        sn = torch.distributions.utils._standard_normal
        eps_t = sn((B, A), torch.float32, self.device)  # target rsample (agent.py:204)
        eps_a = sn((B, A), torch.float32, self.device)  # actor rsample (agent.py:241)
        return idx.reshape(1, B), torch.stack([eps_t, eps_a]).reshape(1, 2, B, A)

    def training_step(self):
        """One SAC gradient step on the engine (agent.py:302-327)."""
        eng = self._engine()
        if self.rng_mode == "reference":
            idx, eps = self._reference_rng_inputs()
            eng.train(self.replay_buffer, 1, indices=idx, eps=eps)
        else:
            self.replay_buffer._check(self.config["train"]["batch_size"])
            eng.train(self.replay_buffer, 1)

    def train_steps(self, n: int) -> None:
        """n consecutive gradient steps (device RNG) replayed from a hipGraph."""
        eng = self._engine()
        if self.rng_mode == "reference":
            for _ in range(n):
                self.training_step()
        else:
            self.replay_buffer._check(self.config["train"]["batch_size"])
            eng.train_graph(self.replay_buffer, n, self.graph_chunk)

    def _loss_log(self, active_logger) -> Optional[LossLog]:
        """logger.log_losses_every (default 1000 gradient steps; 0 = off)."""
        every = int(self.config["logger"].get("log_losses_every", 1000))
        if active_logger is None or self.engine is None or every <= 0 or not hasattr(active_logger, "log_scalar"):
            return None
        return LossLog(self.engine, active_logger, every)

    def _q_log(self, active_logger) -> Optional[QValueLog]:
        """logger.log_q_values: per-env-step Q values, flushed every
        logger.q_values_flush_every env steps (default 256) without host syncs."""
        if active_logger is None or not self.config["logger"]["log_q_values"]:
            return None
        return QValueLog(self, active_logger, int(self.config["logger"].get("q_values_flush_every", 256)))

    def last_losses(self) -> Dict[str, float]:
        """Losses of the last step (reads device memory: synchronises)."""
        l = self._engine().losses()
        return {"q1_loss": l[0], "q2_loss": l[1], "policy_loss": l[2], "alpha_loss": l[3],
                "alpha": float(self.alpha.item())}

    # Reference sub-steps (agent.py:195-300), unfused.  training_step() runs
    # them fused on the HIP engine; called one by one they keep the reference's
    # semantics on the engine's own state: the modules' parameters, the Adam
    # moments and log alpha ARE the engine's buffers, so these run as PyTorch
    # eager ops on the GPU (the reference's own code, not the hot path), with
    # the optimizer step counts taken from and returned to the engine and the
    # packed MFMA copies re-derived after each update (sync_params).
    # tests/test_gpu_substeps.py: the five composed == one fused step.
    def _opt_step(self, opt, idx: int) -> None:
        eng = self._engine()
        t = float(eng.opt_steps[idx].item())
        for st in opt.state.values():
            st["step"] = torch.tensor(t)
        opt.step()
        eng.opt_steps[idx] = t + 1.0

    def compute_target_q_values(self, rewards: Any, dones: Any, next_states: Any) -> Any:
        """y = r + gamma (1 - d)(min Q_t(s', a') - alpha log pi(a'|s')) (agent.py:195-211)."""
        self._engine()
        with torch.no_grad():
            alpha = self.alpha.detach()
            next_actions, next_log_pi = self.policy_net.sample_action(next_states)
            q1 = self.q_net1_target(next_states, next_actions)
            q2 = self.q_net2_target(next_states, next_actions)
            return rewards + self.config["sac"]["gamma"] * (1 - dones) * (torch.min(q1, q2) - alpha * next_log_pi)

    def update_q_networks(self, states: Any, actions: Any, target_q_values: Any) -> None:
        """MSE critic losses, one Adam step per critic (agent.py:213-236)."""
        eng = self._engine()
        for net, opt, idx in ((self.q_net1, self.q1_optimizer, 1), (self.q_net2, self.q2_optimizer, 2)):
            loss = torch.nn.functional.mse_loss(net(states, actions), target_q_values)
            opt.zero_grad()
            loss.backward()
            self._opt_step(opt, idx)
        eng.sync_params()

    def update_policy_network(self, states: Any):
        """L_pi = mean(alpha log pi - min Q) through the current critics; returns log pi (agent.py:238-260)."""
        eng = self._engine()
        actions, log_pi = self.policy_net.sample_action(states)
        min_q = torch.min(self.q_net1(states, actions), self.q_net2(states, actions))
        policy_loss = (self.alpha.detach() * log_pi - min_q).mean()
        self.policy_optimizer.zero_grad()
        policy_loss.backward()
        self._opt_step(self.policy_optimizer, 0)
        for net in (self.q_net1, self.q_net2):  # the reference leaves critic grads behind; drop them
            net.zero_grad(set_to_none=True)
        eng.sync_params()
        return log_pi

    def update_entropy_temperature(self, log_pi: Any) -> Dict[str, float]:
        """Adam step on float64 log alpha (agent.py:263-280); {} when alpha is fixed."""
        eng = self._engine()
        if not self._auto:
            return {}
        term = (log_pi + self.target_entropy).detach()
        alpha_loss = -(self.log_alpha.to(term.dtype) * term).mean()
        if eng.alpha_updates:  # off after a reference-style load_agent (agent.py:550-554)
            self.log_alpha.grad = (-term.mean()).to(self.log_alpha.dtype).reshape(self.log_alpha.shape)
            self._opt_step(self.alpha_optimizer, 3)
            self.log_alpha.grad = None
            eng.alpha_state[1] = eng.alpha_state[0].exp()
        return {"alpha_loss": alpha_loss.item(), "alpha": self.alpha.item()}

    def soft_update_target_networks(self) -> None:
        """Polyak t <- tau p + (1 - tau) t (agent.py:282-300)."""
        eng = self._engine()
        tau = self.config["sac"]["tau"]
        with torch.no_grad():
            for tgt, src in ((self.q_net1_target, self.q_net1), (self.q_net2_target, self.q_net2)):
                for tp, sp in zip(tgt.parameters(), src.parameters()):
                    tp.data.copy_(tau * sp.data + (1.0 - tau) * tp.data)
        eng.sync_params()

    # ------------------------------------------------------------------ loops
    def run_training_loop(self, num_episodes: int, logger=None, tqdm_disable: bool = False,
                          print_rewards: bool = False) -> Dict[str, float]:
        active_logger = logger or self.logger
        total_episodes = total_steps = 0
        returns_window = deque(maxlen=100)
        best_avg_return = -float("inf")
        avg_return = float("nan")
        tr = self.config["train"]
        update_every = tr.get("update_frequency", 1)
        n_grad = tr.get("gradient_steps_per_update", 1)
        loss_log = self._loss_log(active_logger)
        q_log = self._q_log(active_logger)
        for episode in _tqdm(range(num_episodes), disable=tqdm_disable):
            state, _ = self.env.reset()
            done = False
            episode_return = 0.0
            total_episodes += 1
            episode_steps = 0
            while not done:
                action = self.select_action(state)
                next_state, reward, terminated, truncated, _ = self.env.step(action)
                done = terminated or truncated
                self.store_transition(state, action, reward, next_state, done)
                state = next_state
                episode_return += reward
                episode_steps += 1
                total_steps += 1
                if self.can_update() and total_steps % update_every == 0:
                    self._run_updates(n_grad)
                    if loss_log is not None:
                        loss_log.after_updates(total_steps)
                if q_log is not None:  # Q(s', a) of this env step (agent.py:370-376), no host sync
                    q_log.record(state, action, total_steps)
            returns_window.append(episode_return)
            avg_return = float(np.mean(returns_window))
            best_avg_return = max(best_avg_return, avg_return)
            if active_logger is not None and self.config["logger"]["log_episode_stats"]:
                active_logger.log_episode_metrics(episode_idx=episode, reward=episode_return, length=episode_steps)
            if print_rewards:
                print(f"Episode {episode}, Return: {episode_return:.2f}, "
                      f"Average Return(last 100 episodes): {avg_return:.2f}")
        if self.engine is not None:
            self.engine.check()
        if loss_log is not None:
            loss_log.finish()
        if q_log is not None:
            q_log.finish()
        metrics = {"total_episodes": total_episodes, "best_avg_return": best_avg_return,
                   "final_avg_return": avg_return}
        if active_logger is not None:
            active_logger.log_hparams(self.config, metrics)
        if self.config["logger"]["save_model"]["enabled"]:
            save_path = self.config["logger"]["save_model"]["path"]
            if save_path is None:
                save_path = active_logger.run_dir
            else:
                os.makedirs(save_path, exist_ok=True)
            model_path = os.path.join(save_path, "sac_agent.pth")
            self.save_agent(model_path)
            print(f"Agent saved to {model_path}")
        if active_logger is not None and self.config["logger"]["log_episode_stats"]:
            from .utils.logger_utils import save_lengths, save_rewards

            save_rewards(active_logger.run_dir, active_logger.episode_rewards)
            save_lengths(active_logger.run_dir, active_logger.episode_lengths)
        return metrics

    def run_vectorized_training_loop(self, total_env_steps: int, vec_env: Any = None, logger=None,
                                     tqdm_disable: bool = True, print_rewards: bool = False,
                                     seed: Optional[int] = None,
                                     callback: Optional[Callable[[Dict[str, float]], None]] = None) -> Dict[str, float]:
        """Batched form of ``run_training_loop`` (agent.py:329-418) over a
        ``SyncVectorEnv`` of N envs.

        Per vector step: ONE policy kernel for the N actions, the N env steps on
        the host, ONE push of the N transitions, then every gradient step that
        fell due in those N env steps (``update_frequency`` /
        ``gradient_steps_per_update``, counted per env step exactly as the
        reference counts them) as ONE engine call: K steps per launch sequence,
        hipGraph replay when K >= graph_chunk, no host synchronisation.  With
        N = 1 it performs the reference loop's exact sequence of pushes,
        updates and RNG draws (tests/test_gpu_rollout.py).

        ``vec_env`` defaults to ``self.env`` (pass a ``SyncVectorEnv`` as the
        agent's env so ``_set_seed`` seeds env i with seed + i).  Stops after the
        first vector step that reaches ``total_env_steps``.

        ``callback`` (optional) is called after every vector step with the
        loop's host counters (``env_steps``, ``gradient_steps``, ``episodes``,
        ``avg_return`` over the last 100 episodes): the hook of
        ``sac.replicas.ReplicaAggregator`` (independent-seed replicas, one per
        GPU, sac/train_replicas.py).  It must not synchronise the device."""
        env = vec_env if vec_env is not None else self.env
        if not hasattr(env, "num_envs"):
            raise TypeError("run_vectorized_training_loop needs a vectorised env (sac.vector_env.SyncVectorEnv)")
        active_logger = logger or self.logger
        tr = self.config["train"]
        update_every = tr.get("update_frequency", 1)
        n_grad = tr.get("gradient_steps_per_update", 1)
        N = env.num_envs
        obs, _ = env.reset(seed=seed)
        ep_ret = np.zeros(N, np.float64)
        ep_len = np.zeros(N, np.int64)
        returns_window = deque(maxlen=100)
        best_avg_return = -float("inf")
        avg_return = float("nan")
        total_steps = total_episodes = grad_steps = 0
        log_episodes = active_logger is not None and self.config["logger"]["log_episode_stats"]
        loss_log = self._loss_log(active_logger)
        q_log = self._q_log(active_logger)
        pbar = _tqdm(range((int(total_env_steps) + N - 1) // N), disable=tqdm_disable)
        for _ in pbar:
            actions = self.select_actions(obs)
            next_obs, rewards, terminated, truncated, info = env.step(actions)
            dones = np.logical_or(terminated, truncated)
            len_before = len(self.replay_buffer)
            self.store_transitions(obs, actions, rewards, info["final_obs"], dones)
            old = total_steps
            total_steps += N
            due = due_updates_gated(old, total_steps, len_before, self.replay_buffer.capacity,
                                    tr["warming_steps"], update_every, n_grad)
            if self.can_update() and due:
                self._run_updates(due)
                grad_steps += due
                if loss_log is not None:
                    loss_log.after_updates(total_steps)
            if q_log is not None:  # env step old + 1 + i logs Q(s'_i, a_i) under the critics after this vector step
                q_log.record(info["final_obs"], actions, old + 1)
            ep_ret += rewards
            ep_len += 1
            for i in np.nonzero(dones)[0]:
                returns_window.append(float(ep_ret[i]))
                avg_return = float(np.mean(returns_window))
                best_avg_return = max(best_avg_return, avg_return)
                if log_episodes:
                    active_logger.log_episode_metrics(episode_idx=total_episodes, reward=float(ep_ret[i]),
                                                      length=int(ep_len[i]))
                if print_rewards:
                    print(f"Episode {total_episodes}, Return: {ep_ret[i]:.2f}, "
                          f"Average Return(last 100 episodes): {avg_return:.2f}")
                total_episodes += 1
                ep_ret[i] = 0.0
                ep_len[i] = 0
            obs = next_obs
            if callback is not None:
                callback({"env_steps": total_steps, "gradient_steps": grad_steps, "episodes": total_episodes,
                          "avg_return": avg_return})
        if self.engine is not None:
            self.engine.check()  # a timed-out hand-off invalidates the run: raise, do not report it
        if loss_log is not None:
            loss_log.finish()
        if q_log is not None:
            q_log.finish()
        metrics = {"total_episodes": total_episodes, "best_avg_return": best_avg_return,
                   "final_avg_return": avg_return, "total_env_steps": total_steps, "gradient_steps": grad_steps}
        if active_logger is not None:
            active_logger.log_hparams(self.config, metrics)
        return metrics

    def eval_agent(self, num_episodes: int, render_mode: Optional[str] = None, tqdm_disable: bool = False,
                   print_returns: bool = False, writer=None) -> float:
        eval_env = self._get_render_environment(render_mode)
        total_return = 0.0
        for episode in _tqdm(range(num_episodes), disable=tqdm_disable):
            state, _ = eval_env.reset()
            done = False
            episode_return = 0.0
            length = 0
            while not done:
                action = self.select_action(state, deterministic=True)
                next_state, reward, terminated, truncated, _ = eval_env.step(action)
                done = terminated or truncated
                state = next_state
                episode_return += reward
                length += 1
            total_return += episode_return
            if print_returns:
                print(f"Evaluation Episode {episode}, Return: {episode_return:.2f}")
            if writer is not None:
                writer.add_scalar("Eval/Episode/Return", episode_return, episode)
                writer.add_scalar("Eval/Episode/Length", length, episode)
        avg_return = total_return / num_episodes
        if print_returns:
            print(f"Average Return over {num_episodes} episodes: {avg_return:.2f}")
        if eval_env is not self.env:
            eval_env.close()
        return avg_return

    def _get_render_environment(self, render_mode: Optional[str]):
        if render_mode is None or getattr(self.env, "render_mode", None) == render_mode:
            return self.env
        spec = getattr(self.env, "spec", None)
        if spec is not None and getattr(spec, "id", None):
            try:
                import gymnasium as gym

                print(f"Creating new environment for evaluation with render_mode='{render_mode}'")
                eval_env = gym.make(spec.id, render_mode=render_mode)
                seed = self.config["train"].get("seed")
                if seed is not None:
                    eval_env.reset(seed=seed)
                    eval_env.action_space.seed(seed)
                return eval_env
            except Exception as e:  # noqa: BLE001 - same behaviour as the reference
                print(f"Warning: Failed to create new env for rendering: {e}. Using original env.")
                return self.env
        print("Warning: Cannot create new env for rendering as env.spec.id is not available. Using original env.")
        return self.env

    def _log_q_values(self, states: Any, actions: Any, logger, step: int) -> None:
        with torch.no_grad():
            q1 = self.q_net1(states, actions)
            q2 = self.q_net2(states, actions)
            logger.log_q_values(q1.mean().item(), q2.mean().item(), step)

    def _infer_env_name(self, env) -> str:
        spec = getattr(env, "spec", None)
        if spec is not None and getattr(spec, "id", None):
            return spec.id
        return env.__class__.__name__

    def show_config(self, indent: int = 4) -> None:
        pprint.PrettyPrinter(indent=indent).pprint(self.config)

    def print_net_architectures(self) -> None:
        print("Policy Network Architecture:")
        print(self.policy_net)
        print("\nQ-Network 1 Architecture:")
        print(self.q_net1)
        print("\nQ-Network 2 Architecture:")
        print(self.q_net2)

    # ------------------------------------------------------------------ checkpoints
    def _export_steps(self) -> None:
        if self.engine is None:
            return
        steps = self.engine.opt_steps.cpu().tolist()
        for opt, i in ((self.policy_optimizer, 0), (self.q1_optimizer, 1), (self.q2_optimizer, 2),
                       (self.alpha_optimizer, 3)):
            if opt is None:
                continue
            for st in opt.state.values():
                st["step"] = torch.tensor(float(steps[i]))

    def save_agent(self, filepath: str) -> None:
        """Same checkpoint dict as the reference (agent.py:521-536).  Raises
        HandoffTimeout instead of saving a state an invalid step produced."""
        if self.engine is not None:
            self.engine.check()
        self._export_steps()
        ckpt = {
            "policy_net_state_dict": self.policy_net.state_dict(),
            "q_net1_state_dict": self.q_net1.state_dict(),
            "q_net2_state_dict": self.q_net2.state_dict(),
            "q_net1_target_state_dict": self.q_net1_target.state_dict(),
            "q_net2_target_state_dict": self.q_net2_target.state_dict(),
            "policy_optimizer_state_dict": self.policy_optimizer.state_dict(),
            "q1_optimizer_state_dict": self.q1_optimizer.state_dict(),
            "q2_optimizer_state_dict": self.q2_optimizer.state_dict(),
        }
        if self._auto:
            ckpt["log_alpha"] = self.log_alpha.detach().clone()
            ckpt["alpha_optimizer_state_dict"] = self.alpha_optimizer.state_dict()
        torch.save(ckpt, filepath)

    def _import_opt(self, opt, sd, key: Optional[str], step_idx: int) -> None:
        """Load a torch Adam state_dict into the engine-owned moment buffers."""
        eng = self.engine
        params = list(opt.param_groups[0]["params"])
        for g, gsd in zip(opt.param_groups, sd["param_groups"]):
            for k, v in gsd.items():
                if k != "params":
                    g[k] = v
        steps = []
        for i, p in enumerate(params):
            st = sd["state"].get(i)
            cur = opt.state[p]
            if st is None:
                cur["exp_avg"].zero_()
                cur["exp_avg_sq"].zero_()
                steps.append(0.0)
                continue
            cur["exp_avg"].copy_(st["exp_avg"].reshape(cur["exp_avg"].shape))
            cur["exp_avg_sq"].copy_(st["exp_avg_sq"].reshape(cur["exp_avg_sq"].shape))
            steps.append(float(st["step"]))
        if eng is not None and steps:
            eng.opt_steps[step_idx] = max(steps)

    def load_agent(self, filepath: str) -> None:
        """Load a reference-format checkpoint (agent.py:538-554).

        Loaded with ``weights_only=True``: checkpoints are plain tensors/dicts."""
        ckpt = torch.load(filepath, map_location=self.device, weights_only=True)
        self.policy_net.load_state_dict(ckpt["policy_net_state_dict"])
        self.q_net1.load_state_dict(ckpt["q_net1_state_dict"])
        self.q_net2.load_state_dict(ckpt["q_net2_state_dict"])
        self.q_net1_target.load_state_dict(ckpt["q_net1_target_state_dict"])
        self.q_net2_target.load_state_dict(ckpt["q_net2_target_state_dict"])
        if self.engine is None:
            self.policy_optimizer.load_state_dict(ckpt["policy_optimizer_state_dict"])
            self.q1_optimizer.load_state_dict(ckpt["q1_optimizer_state_dict"])
            self.q2_optimizer.load_state_dict(ckpt["q2_optimizer_state_dict"])
            return
        self._import_opt(self.policy_optimizer, ckpt["policy_optimizer_state_dict"], "pi", 0)
        self._import_opt(self.q1_optimizer, ckpt["q1_optimizer_state_dict"], "q1", 1)
        self._import_opt(self.q2_optimizer, ckpt["q2_optimizer_state_dict"], "q2", 2)
        if self._auto and "log_alpha" in ckpt:
            la = ckpt["log_alpha"].detach().to(torch.float64).reshape(())
            self.engine.alpha_state[0] = la
            self.engine.alpha_state[1] = la.exp()
            if "alpha_optimizer_state_dict" in ckpt:
                self._import_opt(self.alpha_optimizer, ckpt["alpha_optimizer_state_dict"], None, 3)
            # The reference rebinds self.log_alpha to the checkpoint's tensor but
            # leaves alpha_optimizer bound to the old one (agent.py:550-554): from
            # here on its steps still compute L_alpha, but log_alpha, alpha and the
            # alpha optimizer state stay as loaded.  Reproduced by default
            # (pinned by tests/golden/ref_ckpt_*.npz); train.alpha_after_load:
            # "tune" keeps tuning the loaded log_alpha instead.
            mode = self.config["train"].get("alpha_after_load", "reference")
            if mode not in ("reference", "tune"):
                raise ValueError("train.alpha_after_load must be 'reference' or 'tune'")
            self.engine.set_alpha_update(mode == "tune")
        self.engine.sync_params()
