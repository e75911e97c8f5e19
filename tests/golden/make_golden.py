"""Generate the golden parity fixtures from the *reference* SAC implementation.

Run in the build container only (the reference lives at /root/reference and never
travels to the GPU box):

    python tests/golden/make_golden.py

What it does (capture recipe):
  * stubs ``gymnasium`` and ``torch.utils.tensorboard`` (absent here), imports
    ``sac.agent.SAC`` from /root/reference and builds it on a fake env with the
    requested obs/act widths, ``device='cpu'``, logger disabled;
  * replaces the instance's ``sample_batch`` (reference sac/agent.py:166-193) by a
    fixed seeded batch and ``torch.distributions.normal._standard_normal`` by a
    queue of pre-drawn eps tensors (first pop = target eps, second = actor eps;
    reference sac/models.py:79-87 via torch Normal.rsample);
  * wraps ``torch.Tensor.backward`` to record, in order, L_Q1, L_Q2, L_pi, L_alpha
    (reference sac/agent.py:230, 234, 256, 274) and ``compute_target_q_values`` /
    ``update_policy_network`` to record y and log_pi;
  * after each ``training_step()`` (sac/agent.py:302-327) dumps every state dict,
    the Adam states and log_alpha.

The fixtures are data only (inputs + expected outputs) written with numpy
``savez_compressed``; no reference source is stored.
"""
from __future__ import annotations

import json
import os
import random
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- stubs
def _install_stubs() -> None:
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb

    gym = types.ModuleType("gymnasium")
    gym.Env = object
    gym.make = lambda *a, **k: None
    sys.modules["gymnasium"] = gym


class _Space:
    def __init__(self, n):
        self.shape = (n,)

    def seed(self, s):
        return [s]

    def sample(self):
        return np.zeros(self.shape, np.float32)


class FakeEnv:
    spec = None

    def __init__(self, obs, act):
        self.observation_space = _Space(obs)
        self.action_space = _Space(act)

    def reset(self, seed=None, options=None):
        return np.zeros(self.observation_space.shape, np.float32), {}


def _cfg(c):
    return {
        "sac": {
            "gamma": c.get("gamma", 0.99),
            "tau": c.get("tau", 0.005),
            "alpha": c.get("alpha", 0.1),
            "auto_entropy_tuning": c["auto"],
            "actor_lr": c.get("actor_lr", 3e-4),
            "critic_lr": c.get("critic_lr", 3e-4),
            "alpha_lr": c.get("alpha_lr", 3e-4),
        },
        "q_net": {
            "hidden_sizes": c["q_hidden"],
            "hidden_layers_act": c.get("q_act", "relu"),
            "output_activation": c.get("q_out_act", "identity"),
        },
        "policy_net": {
            "hidden_sizes": c["pi_hidden"],
            "hidden_layers_act": c.get("pi_act", "relu"),
            "output_activation": c.get("pi_out_act", "identity"),
            "log_std_min": c.get("log_std_min", -20),
            "log_std_max": c.get("log_std_max", 2),
            "action_scale": c.get("action_scale", 1.0),
        },
        "buffer": {"capacity": 1000},
        "train": {
            "gradient_steps_per_update": 1,
            "seed": c.get("seed", 0),
            "batch_size": c["batch"],
            "warming_steps": 10,
            "device": "cpu",
        },
        "logger": {
            "enabled": False,
            "log_dir": "runs",
            "env_name": "Fake",
            "agent_name": "SAC",
            "run_name": "g",
            "use_timestamp": False,
            "timestamp_format": "%Y",
            "flush_secs": 10,
            "log_episode_stats": False,
            "log_q_values": False,
            "save_model": {"enabled": False, "path": None},
        },
    }


CONFIGS = {
    # C1 (BASELINE configs[0]): InvertedPendulum-shaped plumbing config.
    "c1_fixed": dict(obs=4, act=1, q_hidden=[64, 64], pi_hidden=[64, 64], batch=64,
                     auto=False, steps=3, full=True),
    "c1_auto": dict(obs=4, act=1, q_hidden=[64, 64], pi_hidden=[64, 64], batch=64,
                    auto=True, steps=3, full=True),
    # ELU, three hidden layers with a 16-wide one (padding), tight log_std clamp
    # so the clamp gradient mask is exercised, action_scale != 1.
    "elu3_clamp": dict(obs=6, act=2, q_hidden=[32, 32, 16], pi_hidden=[32, 32, 16],
                       q_act="elu", pi_act="elu", batch=32, auto=True, steps=3,
                       log_std_min=-0.05, log_std_max=0.05, action_scale=2.0,
                       full=True, seed=3),
    "mix_act": dict(obs=5, act=3, q_hidden=[40, 24], pi_hidden=[24, 40],
                    q_act="leaky_relu", pi_act="selu", batch=48, auto=False,
                    gamma=0.9, tau=0.01, alpha=0.2, steps=3, full=True, seed=7),
    "gelu_tanh": dict(obs=3, act=2, q_hidden=[32, 32], pi_hidden=[32, 32],
                      q_act="gelu", pi_act="tanh", batch=32, auto=True, steps=3,
                      full=True, seed=11, alpha=0.05, actor_lr=1e-3,
                      critic_lr=2e-3, alpha_lr=5e-3),
    # ConstantRewardEnv semantics (reference sac/envs.py:15-46): r=1, every
    # transition terminal => y == r exactly.
    "const_reward": dict(obs=1, act=1, q_hidden=[64, 64], pi_hidden=[64, 64],
                         batch=64, auto=False, steps=2, full=True, force_done=1.0,
                         force_reward=1.0),
    # C2 (BASELINE configs[1]): BipedalWalker shape, auto-alpha as
    # hparam_search/configs/bipedal_walker.yaml:8.
    "c2": dict(obs=24, act=4, q_hidden=[256, 256], pi_hidden=[256, 256], batch=256,
               auto=True, steps=3, full_steps=[1]),
    # donkey_car_new.yaml shape: [256,256,32] ELU, B=128, tau .02, lr 4e-4.
    "donkey_new": dict(obs=32, act=2, q_hidden=[256, 256, 32],
                       pi_hidden=[256, 256, 32], q_act="elu", pi_act="elu",
                       batch=128, auto=False, tau=0.02, actor_lr=4e-4,
                       critic_lr=4e-4, steps=2, full_steps=[], seed=23),
}


def _summary(t: np.ndarray) -> np.ndarray:
    """[sum, sum of squares, 64 strided samples] in float64."""
    f = t.astype(np.float64).ravel()
    idx = np.linspace(0, f.size - 1, num=min(64, f.size)).astype(np.int64)
    samp = np.zeros(64)
    samp[: idx.size] = f[idx]
    return np.concatenate([[f.sum(), (f * f).sum()], samp])


def _state(agent, want_full: bool, prefix: str, out: dict) -> None:
    nets = {
        "policy": agent.policy_net,
        "q1": agent.q_net1,
        "q2": agent.q_net2,
        "q1t": agent.q_net1_target,
        "q2t": agent.q_net2_target,
    }
    for nname, net in nets.items():
        for k, v in net.state_dict().items():
            arr = v.detach().cpu().numpy().astype(np.float32)
            key = f"{prefix}/{nname}/{k}"
            out[key if want_full else key + "#summary"] = arr if want_full else _summary(arr)
    opts = {"opt_policy": agent.policy_optimizer, "opt_q1": agent.q1_optimizer,
            "opt_q2": agent.q2_optimizer}
    if getattr(agent, "alpha_optimizer", None) is not None:
        opts["opt_alpha"] = agent.alpha_optimizer
    for oname, opt in opts.items():
        sd = opt.state_dict()
        for pid, st in sd["state"].items():
            for field in ("exp_avg", "exp_avg_sq"):
                arr = st[field].detach().cpu().numpy()
                arr = arr.astype(np.float64 if oname == "opt_alpha" else np.float32)
                key = f"{prefix}/{oname}/{pid}/{field}"
                out[key if want_full else key + "#summary"] = arr if want_full else _summary(arr)
            out[f"{prefix}/{oname}/{pid}/step"] = np.array(float(st["step"]), np.float64)
    if getattr(agent, "log_alpha", None) is not None:
        out[f"{prefix}/log_alpha"] = np.array(agent.log_alpha.item(), np.float64)
    out[f"{prefix}/alpha"] = np.array(float(agent.alpha.item()), np.float64)


def _draw_inputs(rng, c) -> dict:
    """One step's injected batch + eps (the fixtures' seeded draw order)."""
    B, O, A = c["batch"], c["obs"], c["act"]
    s = rng.standard_normal((B, O)).astype(np.float32)
    a = rng.uniform(-1, 1, (B, A)).astype(np.float32)
    r = rng.standard_normal(B).astype(np.float32)
    s2 = rng.standard_normal((B, O)).astype(np.float32)
    d = (rng.random(B) < 0.05).astype(np.float32)
    if "force_done" in c:
        d[:] = c["force_done"]
    if "force_reward" in c:
        r[:] = c["force_reward"]
    eps_t = rng.standard_normal((B, A)).astype(np.float32)
    eps_a = rng.standard_normal((B, A)).astype(np.float32)
    return dict(s=s, a=a, r=r, s2=s2, d=d, eps_t=eps_t, eps_a=eps_a)


def _inject_step(agent, inputs: dict):
    """One reference training_step() (sac/agent.py:302-327) on the given batch
    and eps; returns (losses [4] float64, y, log_pi)."""
    import torch.distributions.normal as tdn
    from collections import namedtuple

    T = namedtuple("Transition", ("state", "action", "reward", "next_state", "done"))
    batch = T(*(torch.from_numpy(inputs[k]) for k in ("s", "a", "r", "s2", "d")))
    agent.sample_batch = lambda b=batch: b
    queue = [torch.from_numpy(inputs["eps_t"].copy()), torch.from_numpy(inputs["eps_a"].copy())]

    def fake_sn(shape, dtype, device, q=queue):
        e = q.pop(0)
        assert tuple(e.shape) == tuple(shape), (e.shape, shape)
        return e.to(dtype=dtype, device=device)

    recorded: list = []
    orig_backward = torch.Tensor.backward

    def rec_backward(self, *a, **k):
        recorded.append(float(self.detach().double().item()))
        return orig_backward(self, *a, **k)

    cap = {}
    orig_ctq = type(agent).compute_target_q_values
    orig_upn = type(agent).update_policy_network

    def ctq(self, *a_, **k_):
        y = orig_ctq(self, *a_, **k_)
        cap["y"] = y.detach().numpy().copy()
        return y

    def upn(self, *a_, **k_):
        lp = orig_upn(self, *a_, **k_)
        cap["log_pi"] = lp.detach().numpy().copy()
        return lp

    agent.compute_target_q_values = types.MethodType(ctq, agent)
    agent.update_policy_network = types.MethodType(upn, agent)
    orig_sn = tdn._standard_normal
    tdn._standard_normal = fake_sn
    torch.Tensor.backward = rec_backward
    try:
        agent.training_step()
    finally:
        torch.Tensor.backward = orig_backward
        tdn._standard_normal = orig_sn
    assert not queue, "eps queue not fully consumed"
    losses = recorded + ([np.nan] if len(recorded) == 3 else [])
    return np.array(losses, np.float64), cap["y"], cap["log_pi"]


def capture(name: str, c: dict) -> dict:
    from sac.agent import SAC  # reference, imported after stubs
    import sac.models  # noqa: F401

    cfg = _cfg(c)
    agent = SAC(FakeEnv(c["obs"], c["act"]), cfg)
    out: dict = {"config": np.array(json.dumps({"name": name, **c, "cfg": cfg}))}
    full_steps = c.get("full_steps", list(range(1, c["steps"] + 1)) if c.get("full") else [])
    _state(agent, bool(c.get("full")) or 0 in full_steps, "init", out)

    rng = np.random.default_rng(123 + sum(map(ord, name)))
    for step in range(1, c["steps"] + 1):
        inputs = _draw_inputs(rng, c)
        for k_, v_ in inputs.items():
            out[f"step{step}/in/{k_}"] = v_
        losses, y, log_pi = _inject_step(agent, inputs)
        out[f"step{step}/out/losses"] = losses
        out[f"step{step}/out/y"] = y
        out[f"step{step}/out/log_pi"] = log_pi
        _state(agent, step in full_steps, f"step{step}/post", out)
    return out


def capture_replay_sample() -> dict:
    """Pin the reference sampler's RNG consumption (replay_buffer.py:32-39):
    with ``random.seed(s)``, which deque positions does ``sample`` return?"""
    from sac.replay_buffer import ReplayBuffer

    out = {}
    for cap, n_push, B, seed in [(100, 60, 16, 0), (100, 250, 32, 1), (5000, 5000, 256, 2),
                                 (1000, 1500, 64, 3)]:
        rb = ReplayBuffer(cap)
        for i in range(n_push):
            rb.push(np.array([i], np.float32), np.array([0.0], np.float32), float(i),
                    np.array([i + 1], np.float32), False)
        random.seed(seed)
        got = rb.sample(B)
        out[f"cap{cap}_n{n_push}_b{B}_s{seed}"] = np.array([t.reward for t in got], np.float64)
    return out


def capture_checkpoint() -> dict:
    """the reference's own checkpoint round trip (agent.py:521-554).

    Agent A (c1_auto config, seed 0) runs 2 injected steps and writes
    ``ref_ckpt_c1_auto.pth`` with the reference's save_agent (committed next to
    this script: a file the reference itself wrote, loaded by the tests with
    torch.load(weights_only=True)).  Then
      cont/: A continues with steps 3 and 4 (no reload);
      load/: a FRESH agent B (seed 5: different init) runs the reference's
             load_agent on that file and steps 3 and 4 on the same inputs.
    B's log_alpha stays at the loaded value: load_agent rebinds log_alpha but
    not alpha_optimizer (agent.py:550-554), so B's alpha steps update an orphan.
    Full post-step state is stored for both."""
    from sac.agent import SAC

    c = dict(CONFIGS["c1_auto"])
    out = {"config": np.array(json.dumps({"name": "ref_ckpt", **c, "cfg": _cfg(c)}))}
    rng = np.random.default_rng(2024)
    inputs = [_draw_inputs(rng, c) for _ in range(4)]
    for k, inp in enumerate(inputs, 1):
        for kk, v in inp.items():
            out[f"step{k}/in/{kk}"] = v
    a = SAC(FakeEnv(c["obs"], c["act"]), _cfg(c))
    _state(a, True, "init", out)
    for k in (1, 2):
        out[f"step{k}/out/losses"] = _inject_step(a, inputs[k - 1])[0]
    _state(a, True, "step2/post", out)
    path = os.path.join(OUT, "ref_ckpt_c1_auto.pth")
    a.save_agent(path)
    b = SAC(FakeEnv(c["obs"], c["act"]), _cfg(dict(c, seed=5)))
    _state(b, True, "fresh_init", out)
    b.load_agent(path)
    for k in (3, 4):
        for tag, ag in (("cont", a), ("load", b)):
            losses, y, lp = _inject_step(ag, inputs[k - 1])
            out[f"{tag}/step{k}/out/losses"] = losses
            out[f"{tag}/step{k}/out/y"] = y
            _state(ag, True, f"{tag}/step{k}/post", out)
    return out


LOOP_CASES = {
    # tag: (warming_steps, update_frequency, gradient_steps_per_update, capacity, episodes)
    "w10_u1_g1": (10, 1, 1, 1000, 9),
    "w13_u3_g2": (13, 3, 2, 1000, 9),
    "w20_u2_g3_cap32": (20, 2, 3, 32, 10),
    "w50_u1_g1_cap40": (50, 1, 1, 40, 8),  # warming_steps > capacity: never updates
}


def capture_loop() -> dict:
    """the reference's run_training_loop (agent.py:329-418) on the
    deterministic DetEnv (tests/golden/det_env.py: observations, rewards and
    episode ends depend only on counters, not on actions).  training_step is
    replaced by a recorder: for every call, the number of transitions pushed so
    far (= the loop's total_steps) and len(replay_buffer).  Also stored: the
    final deque content (state, reward, next_state, done; actions are the
    policy's random draws and are not compared) and the episode count."""
    from sac.agent import SAC

    sys.path.insert(0, OUT)
    from det_env import DetEnv

    out = {}
    c = dict(obs=3, act=2, q_hidden=[16, 16], pi_hidden=[16, 16], batch=8, auto=True)
    for tag, (W, u, g, cap, n_ep) in LOOP_CASES.items():
        cfg = _cfg(c)
        cfg["buffer"]["capacity"] = cap
        cfg["train"].update(warming_steps=W, update_frequency=u, gradient_steps_per_update=g)
        agent = SAC(DetEnv(c["obs"], c["act"]), cfg)
        pushed = [0]
        calls = []
        orig_store = agent.store_transition

        def store(*a_, _o=orig_store, _p=pushed):
            _p[0] += 1
            return _o(*a_)

        agent.store_transition = store
        agent.training_step = lambda _c=calls, _p=pushed, _a=agent: _c.append((_p[0], len(_a.replay_buffer)))
        metrics = agent.run_training_loop(n_ep, tqdm_disable=True)
        mem = list(agent.replay_buffer.memory)
        out[f"{tag}/calls"] = np.array(calls, np.int64).reshape(-1, 2)
        out[f"{tag}/total_steps"] = np.array(pushed[0], np.int64)
        out[f"{tag}/episodes"] = np.array(metrics["total_episodes"], np.int64)
        out[f"{tag}/final_avg_return"] = np.array(metrics["final_avg_return"], np.float64)
        out[f"{tag}/mem_state"] = np.stack([np.asarray(t.state, np.float32) for t in mem])
        out[f"{tag}/mem_reward"] = np.array([t.reward for t in mem], np.float64)
        out[f"{tag}/mem_next_state"] = np.stack([np.asarray(t.next_state, np.float32) for t in mem])
        out[f"{tag}/mem_done"] = np.array([t.done for t in mem], bool)
        out[f"{tag}/config"] = np.array([W, u, g, cap, n_ep], np.int64)
    return out


LOGGER_CFG = {"enabled": True, "env_name": "Det", "agent_name": "SAC", "run_name": "pin", "use_timestamp": False,
              "timestamp_format": "%Y", "flush_secs": 10, "log_episode_stats": True, "log_q_values": True,
              "save_model": {"enabled": False, "path": None}}


def _recording_writer(rec: list):
    class Writer:  # stands in for SummaryWriter: every call, in order, as data
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


def capture_logger(tmp: str) -> dict:
    """the reference ExperimentLogger's writer calls
    (sac/utils/experiment_logger.py:54-148), recorded through a stand-in
    SummaryWriter:
      api/<case>: direct calls -- episode metrics, Q values, log_hparams with
        the full SAC config (nested dicts, lists, None, bools) and metrics,
        a repeated log_hparams (ignored), log_hparams with no metrics
        (placeholder_metric), the log_q_values / log_episode_stats gates off,
        flush / close;
      loop: run_training_loop (agent.py:329-418) on DetEnv with the logger on
        and training_step replaced by a no-op (Q values depend on the policy's
        random actions, so only their tags and steps are compared)."""
    import sac.utils.experiment_logger as xl
    from sac.agent import SAC

    sys.path.insert(0, OUT)
    from det_env import DetEnv

    out = {}
    c = dict(obs=3, act=2, q_hidden=[16, 16], pi_hidden=[16, 16], batch=8, auto=True)
    full_cfg = _cfg(c)
    full_cfg["logger"] = dict(LOGGER_CFG, log_dir=tmp)
    cases = {
        "all_on": dict(LOGGER_CFG),
        "gates_off": dict(LOGGER_CFG, log_q_values=False, log_episode_stats=False),
    }
    orig = xl.SummaryWriter
    try:
        for name, lc in cases.items():
            rec: list = []
            xl.SummaryWriter = _recording_writer(rec)
            lg = xl.ExperimentLogger(dict(lc, log_dir=tmp))
            lg.log_episode_metrics(0, 1.5, 10)
            lg.log_episode_metrics(1, -2.25, 7)
            lg.log_q_values(0.25, -0.5, 3)
            lg.log_q_values(1.0, 2.0, 4)
            lg.log_hparams(full_cfg, {"total_episodes": 2, "best_avg_return": 1.5, "final_avg_return": -0.375})
            lg.log_hparams(full_cfg, {"ignored": 1.0})
            lg.flush()
            lg.close()
            rec.append(["lists", lg.episode_rewards, lg.episode_lengths, lg.q1_values, lg.q2_values])
            out[f"api/{name}"] = rec
            rec2: list = []
            xl.SummaryWriter = _recording_writer(rec2)
            lg2 = xl.ExperimentLogger(dict(lc, log_dir=tmp))
            lg2.log_hparams({"a": {"b": [1, 2], "c": None, "d": True, "e": 2.5, "f": "x"}, "g": 3}, {})
            out[f"api/{name}/empty_metrics"] = rec2
        rec3: list = []
        xl.SummaryWriter = _recording_writer(rec3)
        cfg = _cfg(c)
        cfg["logger"] = dict(LOGGER_CFG, log_dir=tmp)
        cfg["train"].update(warming_steps=10)  # >= the batch: the no-op step stands in for a real one
        agent = SAC(DetEnv(c["obs"], c["act"]), cfg)
        agent.training_step = lambda: None
        metrics = agent.run_training_loop(4, tqdm_disable=True)
        out["loop"] = [[r[0], r[1], r[2], None if r[2].startswith("QValues") else r[3], r[4]]
                       if r[0] == "add_scalar" else r for r in rec3]
        out["loop_metrics"] = {k: float(v) for k, v in metrics.items()}
        out["loop_config"] = cfg
        out["npy_dtypes"] = {f: str(np.load(os.path.join(agent.logger.run_dir, f"episode_{f}.npy")).dtype)
                             for f in ("rewards", "lengths")}
    finally:
        xl.SummaryWriter = orig
    return out


def main() -> None:
    _install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(1)
    only = sys.argv[1:]
    for name, c in CONFIGS.items():
        if only and name not in only:
            continue
        out = capture(name, c)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
        print(name, "losses:", [out[f"step{k}/out/losses"].tolist() for k in range(1, c["steps"] + 1)])
    if not only or "replay" in only:
        np.savez_compressed(os.path.join(OUT, "replay_sample.npz"), **capture_replay_sample())
        print("replay_sample written")
    if not only or "ckpt" in only:
        np.savez_compressed(os.path.join(OUT, "ref_ckpt_c1_auto.npz"), **capture_checkpoint())
        print("ref_ckpt_c1_auto written (+ ref_ckpt_c1_auto.pth from the reference's save_agent)")
    if not only or "loop" in only:
        np.savez_compressed(os.path.join(OUT, "ref_loop.npz"), **capture_loop())
        print("ref_loop written")
    if not only or "logger" in only:
        import tempfile

        with tempfile.TemporaryDirectory() as tmp:
            rec = json.loads(json.dumps(capture_logger(tmp)).replace(tmp, "<log_dir>"))  # run-independent
        with open(os.path.join(OUT, "ref_logger.json"), "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)
        print("ref_logger.json written")


if __name__ == "__main__":
    main()
