"""tests/_ties.py on the CPU: a constructed ReLU tie is found on the row that
holds it, and a tie-free draw leaves no tie on any pass (the GPU parity tests
rely on both to keep the per-element parameter check on every network)."""
import numpy as np

import _ties
from oracle import sac_oracle as O


def _state(obs, act, hidden, seed):
    g = np.random.default_rng(seed)

    def mlp(dims):
        W = [(g.standard_normal((o, i)) * np.sqrt(2.0 / (i + o))).astype(np.float32) for i, o in zip(dims, dims[1:])]
        return O.MLP(W, [np.zeros(o, np.float32) for o in dims[1:]])

    hp = O.SacHyper(alpha=0.1, auto_entropy_tuning=True)
    st = O.SacState.fresh(mlp([obs, *hidden, 2 * act]), mlp([obs + act, *hidden, 1]), mlp([obs + act, *hidden, 1]),
                          hp, act)
    return st, hp


def test_relu_tie_is_found_on_its_row():
    st, _ = _state(5, 2, [16, 16], 0)
    x = np.random.default_rng(1).standard_normal((8, 5)).astype(np.float32)
    assert not _ties.relu_ties(st.pi, x).any()
    # move row 3's first hidden pre-activation of unit 0 to exactly 0
    w = st.pi.W[0][0].astype(np.float64)
    x[3] -= (x[3].astype(np.float64) @ w) / (w @ w) * w
    m = _ties.relu_ties(st.pi, x, rel=1e-6)
    assert m[3] and m.sum() == 1


def test_tie_free_draw_leaves_no_tie():
    obs, act, B, n = 6, 2, 512, 2048
    st, hp = _state(obs, act, [64, 64], 2)
    g = np.random.default_rng(3)
    s = g.standard_normal((n + 1, obs)).astype(np.float32)
    rows = dict(obs=s[:n], next_obs=s[1:], act=g.uniform(-1, 1, (n, act)).astype(np.float32),
                rew=g.standard_normal(n).astype(np.float32), done=(g.random(n) < 0.01).astype(np.float32))
    # a loose threshold so that ties do occur at this size
    rel = 1e-4
    idx, et, ea, bt, outs, redrawn, seen = _ties.tie_free_draw(g, rows, n, B, act, hp, [st], rel=rel)
    assert redrawn > 0 and seen
    assert len(set(idx.tolist())) == B
    ties, ref, _ = _ties.step_ties(st, hp, bt, et, ea, rel=rel)
    assert not ties
    np.testing.assert_array_equal(ref["y"], outs[0][0]["y"])
