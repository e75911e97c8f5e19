"""Actor / critic network definitions (API of reference ``sac/models.py``).

The modules are plain ``torch.nn`` parameter containers with the reference's
construction order, seeding, initialisation and ``state_dict`` keys
(``net.{2i}.weight`` / ``net.{2i}.bias``; activations at odd indices), so
checkpoints written by the reference load unchanged and vice versa.

Their ``forward`` methods are the *eager* definition of the maths, used by code
outside the hot path (Q-value logging, notebooks, user code).  The gradient step
itself never calls them: ``sac.agent.SAC.training_step`` runs the fused HIP kernels
of ``libsac_engine.so`` directly on the parameter storage.

Reference cross-walk:
    QNetwork                      sac/models.py:8-42
    PolicyNetwork                 sac/models.py:45-101
    _ACTIVATIONS                  sac/models.py:104-112
    build_mlp                     sac/models.py:115-149
"""
from __future__ import annotations

import math
from typing import List, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

_ACTIVATIONS = {
    "relu": nn.ReLU,
    "tanh": nn.Tanh,
    "elu": nn.ELU,
    "leaky_relu": nn.LeakyReLU,
    "gelu": nn.GELU,
    "selu": nn.SELU,
    "identity": nn.Identity,
}

# engine activation codes (must match csrc/sac_kernels.hip ``enum Act``)
ACT_CODES = {"identity": 0, "relu": 1, "tanh": 2, "elu": 3, "leaky_relu": 4, "gelu": 5, "selu": 6}


def build_mlp(
    obs_size: int,
    hidden_sizes: Sequence[int],
    action_size: int,
    hidden_activations: str = "relu",
    output_activation: str = "identity",
) -> nn.Sequential:
    """``Linear, act`` pairs from ``obs_size`` through ``hidden_sizes`` to
    ``action_size`` (reference sac/models.py:115-149).

    Raises ``ValueError`` for an empty ``hidden_sizes`` and ``KeyError`` for an
    unknown activation name, as the reference does."""
    if not hidden_sizes:
        raise ValueError("hidden_sizes cannot be empty")
    hidden_cls = _ACTIVATIONS[hidden_activations]
    out_cls = _ACTIVATIONS[output_activation]
    widths = [int(obs_size), *[int(h) for h in hidden_sizes], int(action_size)]
    modules: List[nn.Module] = []
    last = len(widths) - 2
    for i, (fan_in, fan_out) in enumerate(zip(widths[:-1], widths[1:])):
        modules.append(nn.Linear(fan_in, fan_out))
        modules.append(out_cls() if i == last else hidden_cls())
    return nn.Sequential(*modules)


def _xavier_zero_(module: nn.Module) -> None:
    # Same visiting order as the reference (self.modules() pre-order), so the
    # global torch RNG is consumed identically.
    for m in module.modules():
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            nn.init.zeros_(m.bias)


def _linears(seq: nn.Sequential) -> List[nn.Linear]:
    return [m for m in seq if isinstance(m, nn.Linear)]


def _act_name(mod: nn.Module) -> str:
    for name, cls in _ACTIVATIONS.items():
        if type(mod) is cls:
            return name
    raise KeyError(type(mod).__name__)


class QNetwork(nn.Module):
    """Q(s, a) -> [B]; input is ``cat([s, a], -1)`` (reference models.py:8-42)."""

    def __init__(self, obs_size, action_size, hidden_sizes, hidden_activations="relu",
                 output_activation="identity", seed=None):
        super().__init__()
        if seed is not None:
            torch.manual_seed(seed)
        self.obs_size = int(obs_size)
        self.action_size = int(action_size)
        self.hidden_activations = hidden_activations
        self.output_activation = output_activation
        self.net = build_mlp(obs_size + action_size, list(hidden_sizes), 1,
                             hidden_activations, output_activation)
        _xavier_zero_(self)

    def forward(self, state, action):
        return self.net(torch.cat((state, action), dim=-1)).squeeze(-1)

    def save_weights(self, filepath):
        torch.save(self.state_dict(), filepath)

    # engine helpers --------------------------------------------------------
    def linears(self) -> List[nn.Linear]:
        return _linears(self.net)

    def _init_weights_xavier(self):
        _xavier_zero_(self)


class PolicyNetwork(nn.Module):
    """Squashed-Gaussian actor (reference models.py:45-101).

    ``forward`` -> (mu, clamp(log_std)); ``sample_action`` -> (tanh(z)*scale,
    log pi) with the tanh change-of-variables correction; ``deterministic_action``
    -> tanh(mu)*scale."""

    def __init__(self, obs_size, action_size, hidden_sizes, log_std_min=-20, log_std_max=2,
                 seed=None, action_scale=1.0, hidden_activations="relu",
                 output_activation="identity"):
        super().__init__()
        if seed is not None:
            torch.manual_seed(seed)
        self.obs_size = int(obs_size)
        self.action_size = int(action_size)
        self.log_std_min = log_std_min
        self.log_std_max = log_std_max
        self.hidden_activations = hidden_activations
        self.output_activation = output_activation
        self.net = build_mlp(obs_size, list(hidden_sizes), 2 * action_size,
                             hidden_activations, output_activation)
        self.action_scale = action_scale
        _xavier_zero_(self)

    def forward(self, state):
        mu, log_std = self.net(state).chunk(2, dim=-1)
        return mu, log_std.clamp(self.log_std_min, self.log_std_max)

    def sample_action(self, state):
        mu, log_std = self.forward(state)
        std = log_std.exp()
        dist = torch.distributions.Normal(mu, std)
        z = dist.rsample()
        log_prob = dist.log_prob(z).sum(dim=-1)
        log_prob = log_prob - (2.0 * (math.log(2.0) - z - F.softplus(-2.0 * z))).sum(dim=-1)
        return torch.tanh(z) * self.action_scale, log_prob

    def deterministic_action(self, state):
        mu, _ = self.forward(state)
        return torch.tanh(mu) * self.action_scale

    def save_weights(self, filepath):
        torch.save(self.state_dict(), filepath)

    def linears(self) -> List[nn.Linear]:
        return _linears(self.net)

    def _init_weights_xavier(self):
        _xavier_zero_(self)
