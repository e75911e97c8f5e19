"""Summation-order ties of one SAC step, and tie-free batch draws for the
fp32 parity checks (test infrastructure; the oracle is the checker).

A "tie" is a decision of the step that fp32 summation order can flip between
two correct implementations (the numpy oracle and the MFMA kernels):

* a hidden ReLU pre-activation p with |p| <= rel * (|W| |x| + |b|) on a pass
  whose backward runs (pi on s, the critics on (s, a) and, with the UPDATED
  critics, on (s, a~)): the unit's mask for that row, and so a rank-one term
  of every lower layer's dW, follows the sign the sum happened to take
  (profiles/r04_debug_wide512_relu_tie.txt);
* the same on the forward-only passes (pi on s', the targets on (s', a')),
  where the flipped unit moves y by ~|p| only, checked all the same;
* a min-Q near-tie of the actor pass, |q1 - q2| <= rel * (|q1| + |q2|): the
  min's backward routes the row's gradient to the other critic.

Reference: /root/reference/sac/agent.py:195-260 (the passes), sac/models.py:
115-149 (the ReLU stacks).  The parity tests draw each step's indices and eps
until no tie is found, so the per-element parameter check (>= 99.5% within
1e-6) runs on every network at every shape instead of being voided."""
import copy

import numpy as np

from oracle import sac_oracle as O

REL = 1e-7


def relu_ties(mlp, x, rel=REL):
    """Rows of this forward with a hidden ReLU pre-activation within fp32
    summation-order noise of 0 (float64 evaluation), as a boolean mask."""
    h = np.asarray(x, np.float64)
    rows = np.zeros(h.shape[0], bool)
    if mlp.hidden_act != "relu":
        return rows
    for i in range(len(mlp.W) - 1):
        W, b = mlp.W[i].astype(np.float64), mlp.b[i].astype(np.float64)
        p = h @ W.T + b
        rows |= np.any(np.abs(p) <= rel * (np.abs(h) @ np.abs(W).T + np.abs(b)), axis=1)
        h = np.maximum(p, 0.0)
    return rows


def step_ties(st, hp, bt, et, ea, rel=REL):
    """Ties of one oracle training step from state `st` (not mutated) on batch
    `bt` with eps (et, ea).  Returns (ties: dict pass -> boolean row mask, for
    the passes with a tie; the oracle's step result; the post-step state).  The
    post-step state is the oracle reference for a one-step parameter comparison
    from `st`."""
    ties = {}
    s = np.asarray(bt.s, np.float32)
    s2 = np.asarray(bt.s2, np.float32)
    a = np.asarray(bt.a, np.float32)
    pc = hp.policy
    ties["pi(s')"] = relu_ties(st.pi, s2, rel)
    ties["pi(s)"] = relu_ties(st.pi, s, rel)
    a2, _, _ = O.policy_sample(st.pi, s2, et, pc)
    at, _, _ = O.policy_sample(st.pi, s, ea, pc)
    sa2 = np.concatenate([s2, a2], 1)
    ties["q1t(s',a')"] = relu_ties(st.q1t, sa2, rel)
    ties["q2t(s',a')"] = relu_ties(st.q2t, sa2, rel)
    sa = np.concatenate([s, a], 1)
    ties["q1(s,a)"] = relu_ties(st.q1, sa, rel)
    ties["q2(s,a)"] = relu_ties(st.q2, sa, rel)
    post = copy.deepcopy(st)
    ref = O.training_step(post, hp, bt, et, ea)
    # the actor pass runs the UPDATED critics on (s, a~); post.q1 / q2 are
    # those (the actor, alpha and Polyak updates leave the critics as they are)
    sat = np.concatenate([s, at], 1)
    ties["q1(s,a~)"] = relu_ties(post.q1, sat, rel)
    ties["q2(s,a~)"] = relu_ties(post.q2, sat, rel)
    q1v = O.q_forward(post.q1, s, at)[0].astype(np.float64)
    q2v = O.q_forward(post.q2, s, at)[0].astype(np.float64)
    ties["minQ(s,a~)"] = np.abs(q1v - q2v) <= 20 * rel * (np.abs(q1v) + np.abs(q2v)) + 1e-9
    return {k: v for k, v in ties.items() if v.any()}, ref, post


# passes whose ties depend on the row's eps_a alone (a~ = pi(s) sampled with it)
# and on the critics' update, which does not read eps_a: such a row is fixed by
# a fresh eps_a, which leaves every other row's ties as they were
ACTOR_PASSES = ("q1(s,a~)", "q2(s,a~)", "minQ(s,a~)")


def tie_free_draw(g, rows, n_rows, B, A, hp, states, max_rounds=64, rel=REL):
    """Draw B distinct indices and eps (et, ea) from rng `g`, then redraw the
    rows of any tie until the step has no tie from any state in `states`
    (oracle trajectories and/or the engine's own state).  A tie is a (row,
    unit) event (~1 per pass per step at B = 4096), so whole-batch redraws
    would never end.  A row tied on a pass before the actor's gets a fresh
    unused index and fresh eps (this moves the critics' update, so a later
    round can show a new actor-pass tie elsewhere); a row tied on the actor
    pass only (the updated critics on (s, a~), the min-Q) gets a fresh eps_a,
    which the critics' update does not read.  Returns (idx, et, ea, batch,
    [(ref, post) per state], rows redrawn, ties seen: pass -> count)."""
    idx = g.choice(n_rows, size=B, replace=False).astype(np.int32)
    et = g.standard_normal((B, A)).astype(np.float32)
    ea = g.standard_normal((B, A)).astype(np.float32)
    seen, redrawn = {}, 0
    for _ in range(max_rounds):
        bt = O.Batch(rows["obs"][idx], rows["act"][idx], rows["rew"][idx], rows["next_obs"][idx], rows["done"][idx])
        outs, row_tied, actor_tied = [], np.zeros(B, bool), np.zeros(B, bool)
        for st in states:
            ties, ref, post = step_ties(st, hp, bt, et, ea, rel)
            for k, m in ties.items():
                seen[k] = seen.get(k, 0) + int(m.sum())
                if k in ACTOR_PASSES:
                    actor_tied |= m
                else:
                    row_tied |= m
            outs.append((ref, post))
        if not (row_tied.any() or actor_tied.any()):
            return idx, et, ea, bt, outs, redrawn, seen
        r = np.flatnonzero(row_tied)
        if r.size:
            free = np.setdiff1d(np.arange(n_rows, dtype=np.int32), idx)
            idx = idx.copy()
            idx[r] = g.choice(free, size=r.size, replace=False).astype(np.int32)
            et[r] = g.standard_normal((r.size, A)).astype(np.float32)
        ra = np.flatnonzero(row_tied | actor_tied)
        ea[ra] = g.standard_normal((ra.size, A)).astype(np.float32)
        redrawn += int(ra.size)
    raise AssertionError(f"ties remain after {max_rounds} rounds of row redraws (ties seen: {seen})")
