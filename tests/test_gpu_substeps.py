"""The reference's sub-step API on the engine's state (sac/agent.py:195-300):
compute_target_q_values -> update_q_networks -> update_policy_network ->
update_entropy_temperature -> soft_update_target_networks, called one by one
with the reference golden's batch and eps, equals the reference's step (and
therefore the fused engine step) within the fp32 parity tolerances of
tests/test_gpu_parity.py; and the engine's fused step continues correctly from
the state the sub-steps leave (Adam step counts, packed copies, log alpha)."""
import numpy as np
import pytest
import torch

from _fixtures import batch, eps, oracle_state

pytestmark = pytest.mark.gpu


def _queue_eps(et, ea):
    """Feed the two rsample draws (target, then actor) as the reference's capture did."""
    import torch.distributions.normal as tdn

    q = [torch.from_numpy(et.copy()), torch.from_numpy(ea.copy())]
    orig = tdn._standard_normal

    def fake(shape, dtype, device):
        e = q.pop(0)
        assert tuple(e.shape) == tuple(shape)
        return e.to(dtype=dtype, device=device)

    tdn._standard_normal = fake
    return lambda: setattr(tdn, "_standard_normal", orig)


@pytest.mark.parametrize("name", ["c1_auto", "c1_fixed"])
def test_substeps_compose_to_the_reference_step(name):
    from _gpu import make_agent, run_step
    from oracle import sac_oracle as O

    agent, fx, meta, nets = make_agent(name, "fp32")
    st, hp, _, _ = oracle_state(name)
    dev = agent.device
    for k in (1, 2):
        b = batch(fx, k)
        et, ea = eps(fx, k)
        ref = O.training_step(st, hp, b, et, ea)
        s, a, r, s2, d = (torch.from_numpy(np.asarray(x)).to(dev) for x in b)
        restore = _queue_eps(et, ea)
        try:
            y = agent.compute_target_q_values(rewards=r, dones=d, next_states=s2)
            agent.update_q_networks(states=s, actions=a, target_q_values=y)
            log_pi = agent.update_policy_network(states=s)
            out = agent.update_entropy_temperature(log_pi=log_pi)
            agent.soft_update_target_networks()
        finally:
            restore()
        torch.cuda.synchronize()
        np.testing.assert_allclose(y.cpu().numpy(), ref["y"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(log_pi.detach().cpu().numpy(), ref["log_pi"], rtol=1e-4, atol=1e-4)
        if hp.auto_entropy_tuning:
            assert out["alpha_loss"] == pytest.approx(ref["losses"][3], rel=1e-4)
            assert abs(float(agent.engine.alpha_state[0]) - st.log_alpha) <= 1e-7
        else:
            assert out == {}
        for key, net in nets.items():
            want = {"policy": st.pi, "q1": st.q1, "q2": st.q2, "q1t": st.q1t, "q2t": st.q2t}[key]
            for pk, w in want.state_dict().items():
                dd = np.abs(net.state_dict()[pk].detach().cpu().numpy() - w)
                assert np.mean(dd <= 1e-6) >= 0.995, (name, k, key, pk)
                assert dd.max() <= 2 * hp.critic_lr * k + 1e-5
    assert [float(x) for x in agent.engine.opt_steps.cpu()[:3]] == [2.0, 2.0, 2.0]
    # the fused engine step continues from that state (step 3 of the fixture)
    b = batch(fx, 3)
    et, ea = eps(fx, 3)
    ref = O.training_step(st, hp, b, et, ea)
    losses, y, _ = run_step(agent, fx, meta, 3)
    floor = float(np.mean(np.abs(st.alpha * ref["log_pi"])) + np.mean(np.abs(ref["y"]))) + 1e-6
    for i, (g, w) in enumerate(zip(losses, ref["losses"])):
        if np.isnan(w):
            assert np.isnan(g)
        else:
            assert abs(g - w) <= 1e-4 * max(abs(w), floor if i == 2 else 1e-3), (i, g, w)
    agent.engine.check()
