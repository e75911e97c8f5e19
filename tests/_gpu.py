"""GPU-side helpers: build an agent on the fixture's config and feed the
fixture's batches/eps through the C ABI with injected indices."""
import copy

import numpy as np
import torch

from _fixtures import batch, eps, init_state_dicts, load


class FakeSpace:
    def __init__(self, n):
        self.shape = (n,)

    def seed(self, s):
        return [s]

    def sample(self):
        return np.zeros(self.shape, np.float32)


class FakeEnv:
    spec = None

    def __init__(self, obs, act):
        self.observation_space = FakeSpace(obs)
        self.action_space = FakeSpace(act)

    def reset(self, seed=None, options=None):
        return np.zeros(self.observation_space.shape, np.float32), {}


def make_agent(name, precision="fp32", capacity=None):
    from sac.agent import SAC

    fx, meta = load(name)
    cfg = copy.deepcopy(meta["cfg"])
    cfg["train"]["device"] = "cuda"
    cfg["train"]["precision"] = precision
    B = meta["batch"]
    cfg["buffer"]["capacity"] = capacity or B * meta["steps"]
    agent = SAC(FakeEnv(meta["obs"], meta["act"]), cfg)
    sds = init_state_dicts(name)
    nets = {"policy": agent.policy_net, "q1": agent.q_net1, "q2": agent.q_net2, "q1t": agent.q_net1_target,
            "q2t": agent.q_net2_target}
    with torch.no_grad():
        for k, net in nets.items():
            for pk, p in net.state_dict().items():
                p.copy_(torch.from_numpy(np.asarray(sds[k][pk])))
    agent.engine.sync_params()
    for k in range(1, meta["steps"] + 1):
        b = batch(fx, k)
        agent.replay_buffer.push_batch(b.s, b.a, b.r, b.s2, b.d)
    return agent, fx, meta, nets


def run_step(agent, fx, meta, k):
    B, A = meta["batch"], meta["act"]
    idx = torch.arange((k - 1) * B, k * B, dtype=torch.int32).reshape(1, B)
    et, ea = eps(fx, k)
    e = torch.from_numpy(np.stack([et, ea])).reshape(1, 2, B, A)
    agent.engine.train(agent.replay_buffer, 1, indices=idx, eps=e)
    torch.cuda.synchronize()
    st = agent.engine.stats.cpu().numpy()
    return st[:4].astype(np.float64), st[4:4 + B], st[4 + B:4 + 2 * B]
