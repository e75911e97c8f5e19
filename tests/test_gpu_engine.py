"""GPU tests of the engine beyond the single-step oracle parity
(tests/test_gpu_parity.py): replay storage and gather, the device sampler,
the policy kernel, graph replay, multi-step determinism and checkpoints.
Every call goes through libsac_engine.so (C ABI)."""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def lib():
    from sac import _engine as E

    return E.load_library()


def _engine(cfgname="c1", precision="fp32", seed=0, capacity=None, **layout):
    """bench.build_engine with kernel layout overrides (sac_engine_config.layout
    and friends, sac.engine.SacEngine(layout=...)) as keyword arguments."""
    import bench

    c = dict(bench.CONFIGS[cfgname])
    if capacity:
        bench.CONFIGS[cfgname] = dict(c, capacity=capacity)
    try:
        return bench.build_engine(cfgname, precision, seed, DEV, layout=layout or None)
    finally:
        bench.CONFIGS[cfgname] = c


# ---------------------------------------------------------------- replay buffer
@pytest.mark.parametrize("layout", ["records", "soa"])
def test_replay_push_gather_ring_exact(layout):
    """push (single rows, staged) + push_batch with wrap-around; gather by
    logical position == the deque model of replay_buffer.py:12-30 bit-exactly,
    for both storage layouts."""
    from sac.replay_buffer import ReplayBuffer

    O, A, cap = 5, 2, 37
    rng = np.random.default_rng(0)
    rb = ReplayBuffer(cap, device=DEV, stage_rows=8, layout=layout)
    model = []
    for it in range(6):
        n = int(rng.integers(1, 30))
        s = rng.standard_normal((n, O), dtype=np.float32)
        a = rng.standard_normal((n, A), dtype=np.float32)
        r = rng.standard_normal(n).astype(np.float64)  # Python-float rewards in the reference
        s2 = rng.standard_normal((n, O), dtype=np.float32)
        d = rng.random(n) < 0.3
        if it % 2 == 0:
            for i in range(n):
                rb.push(s[i], a[i], float(r[i]), s2[i], bool(d[i]))
        else:
            rb.push_batch(s, a, r.astype(np.float32), s2, d)
        for i in range(n):
            model.append((s[i], a[i], np.float32(r[i]), s2[i], np.float32(d[i])))
        model = model[-cap:]
        assert len(rb) == len(model)
        idx = np.arange(len(model))
        t = rb.gather(idx)
        got = [x.cpu().numpy() for x in t]
        for f in range(5):
            want = np.stack([np.asarray(m[f], np.float32) for m in model])
            assert np.array_equal(got[f].reshape(want.shape), want), (it, f)


def test_replay_sample_api(lib):
    from sac.replay_buffer import ReplayBuffer

    rb = ReplayBuffer(100, device=DEV)
    for i in range(10):
        rb.push(np.full(3, i, np.float32), np.full(1, -i, np.float32), float(i), np.full(3, i + 1, np.float32),
                i == 9)
    with pytest.raises(ValueError, match="Not enough samples"):
        rb.sample(11)
    out = rb.sample(10)
    assert sorted(int(t.state[0]) for t in out) == list(range(10))
    for t in out:
        i = int(t.state[0])
        assert t.reward == float(i) and t.done == (i == 9) and np.all(t.next_state == i + 1)


# ---------------------------------------------------------------- device sampler
@pytest.mark.parametrize("size,batch", [(64, 64), (1000, 256), (1_000_000, 256), (1_000_000, 4096)])
def test_device_sampler_equals_host(lib, size, batch):
    from oracle import sampler_oracle as S
    from sac import _engine as E

    f = lib.sac_debug_sample_indices_host
    f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    state = torch.tensor([size, 0, 0], dtype=torch.int64, device=DEV)
    desc = E.ReplayDesc(0, 0, 0, 0, 0, size, 1, 1, state.data_ptr())
    out = torch.empty(batch, dtype=torch.int32, device=DEV)
    for step in (0, 5, 2**33 + 1):
        E.check(lib.sac_replay_sample_indices(ctypes.byref(desc), batch, 11, step, E.ptr(out),
                                              E.stream_handle(DEV)))
        host = np.zeros(batch, np.int32)
        assert f(size, batch, 11, step, host.ctypes.data) == 0
        dev = out.cpu().numpy()
        assert np.array_equal(dev, host)
        assert np.unique(dev).size == batch and dev.min() >= 0 and dev.max() < size
        if batch <= 256:
            assert dev.tolist() == S.sample_indices(size, batch, 11, step)


def test_in_step_sampler_is_the_exported_sampler(lib):
    """A device-sampled step equals the same step fed the host sampler's
    indices for (seed, rng_step): the step kernels gather exactly those rows."""
    eng, rb, c = _engine("c1", "fp32")
    f = lib.sac_debug_sample_indices_host
    f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    eng.train(rb, 3)  # move off step 0
    snap = eng.snapshot()
    step = int(eng.rng_step.item())
    eng.train(rb, 1)
    a = {k: v.clone() for k, v in eng.state_tensors().items()}
    la = eng.stats.clone()
    eng.restore(snap)
    host = np.zeros(c["batch"], np.int32)
    assert f(len(rb), c["batch"], int(eng.cfg.seed), step, host.ctypes.data) == 0
    # device eps stay on (eps=None): only the index source differs
    eng.train(rb, 1, indices=torch.from_numpy(host).reshape(1, -1))
    for k, v in eng.state_tensors().items():
        assert torch.equal(v, a[k]), k
    assert torch.equal(eng.stats, la)


# ---------------------------------------------------------------- determinism / graphs
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_equals_direct_launches(precision):
    eng, rb, _ = _engine("c1", precision)
    snap = eng.snapshot()
    eng.train(rb, 40)
    a = {k: v.clone() for k, v in eng.state_tensors().items()}
    eng.restore(snap)
    eng.train_graph(rb, 40, chunk=16)  # 2 full chunks + a remainder
    for k, v in eng.state_tensors().items():
        assert torch.equal(v, a[k]), k
    assert int(eng.rng_step.item()) == 40
    eng.check()
    assert eng.opt_steps.cpu().tolist()[:3] == [40.0, 40.0, 40.0]


def test_c2_full_size_many_steps_properties():
    """C2 at full size (1e6-row buffer, B=256, bf16): 300 steps stay finite,
    alpha moves the right way, and Polyak keeps targets between their start
    and the online critics (convex combination, tau = 0.005)."""
    eng, rb, c = _engine("c2", "bf16")
    q1t0 = eng.flat["q1t"].clone()
    eng.train_graph(rb, 300, chunk=50)
    torch.cuda.synchronize()
    eng.check()
    losses = eng.losses()
    assert all(np.isfinite(losses)), losses
    assert int(eng.rng_step.item()) == 300
    # targets moved toward the critics but by far less than the critics moved
    d_t = (eng.flat["q1t"] - q1t0).norm().item()
    d_q = (eng.flat["q1"] - q1t0).norm().item()
    assert 0 < d_t < d_q
    lp = eng.last_log_pi().cpu().numpy()
    y = eng.last_targets().cpu().numpy()
    assert np.all(np.isfinite(lp)) and np.all(np.isfinite(y))


# ---------------------------------------------------------------- policy kernel
def _torch_policy(pi, s, eps):
    mu, log_std = pi(s)
    if eps is None:
        return torch.tanh(mu) * pi.action_scale, None
    std = log_std.exp()
    z = mu + eps * std
    a = torch.tanh(z) * pi.action_scale
    lp = torch.distributions.Normal(mu, std).log_prob(z).sum(-1)
    lp = lp - (2 * (np.log(2.0) - z - torch.nn.functional.softplus(-2 * z))).sum(-1)
    return a, lp


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-5), ("bf16", 3e-2)])
def test_policy_act_matches_torch(precision, tol):
    eng, rb, c = _engine("c2", precision, capacity=1000)
    pi = eng.nets["pi"]
    g = torch.Generator(device="cpu").manual_seed(0)
    for n in (1, 7, 300):
        s = torch.randn(n, c["obs"], generator=g).to(DEV)
        eps = torch.randn(n, c["act"], generator=g).to(DEV)
        with torch.no_grad():
            a_ref, _ = _torch_policy(pi, s, None)
            a2_ref, lp_ref = _torch_policy(pi, s, eps)
        a = eng.policy_act(s)
        a2, lp = eng.policy_act(s, eps, want_log_pi=True)
        assert (a - a_ref).abs().max().item() <= tol
        assert (a2 - a2_ref).abs().max().item() <= tol
        assert ((lp - lp_ref).abs() / lp_ref.abs().clamp_min(1.0)).max().item() <= tol


# ---------------------------------------------------------------- checkpoints
def test_save_load_roundtrip_continues_identically(tmp_path):
    from _gpu import make_agent

    agent, fx, meta, _ = make_agent("c1_auto", "fp32")
    agent.train_steps(5)
    path = os.path.join(tmp_path, "ckpt.pth")
    agent.save_agent(path)
    other, _, _, _ = make_agent("c1_auto", "fp32")
    other.load_agent(path)
    for a, b in ((agent.policy_net, other.policy_net), (agent.q_net1, other.q_net1),
                 (agent.q_net2_target, other.q_net2_target)):
        for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
            assert torch.equal(va, vb), ka
    assert torch.equal(agent.engine.alpha_state[:1], other.engine.alpha_state[:1])
    for k in ("m/pi", "v/q1", "v/q2"):
        assert torch.equal(agent.engine.state_tensors()[k], other.engine.state_tensors()[k]), k
    assert agent.engine.opt_steps[:3].tolist() == other.engine.opt_steps[:3].tolist()
    # the same injected step on both gives the same result
    B, A = meta["batch"], meta["act"]
    idx = torch.arange(B, dtype=torch.int32).reshape(1, B)
    e = torch.randn(1, 2, B, A, generator=torch.Generator().manual_seed(1))
    agent.engine.train(agent.replay_buffer, 1, indices=idx, eps=e)
    other.engine.train(other.replay_buffer, 1, indices=idx, eps=e)
    assert torch.equal(agent.engine.flat["pi"], other.engine.flat["pi"])
    assert torch.equal(agent.engine.stats[:4], other.engine.stats[:4])


# ---------------------------------------------------------------- role-split vs row-tile phase kernels
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_role_split_equals_row_tiles(precision):
    """Phases A/C split into per-network workgroups with in-launch hand-offs give
    the same bits as the one-workgroup-per-row-tile kernels (power-of-two batch:
    the min-Q weights are applied after a unit-seed backward, exactly).  Both
    without the hidden split, which sums in another order (tested vs the oracle)."""
    out = {}
    for roles in ("1", "0"):
        eng, rb, c = _engine("c2", precision, capacity=5000, layout="roles" if roles == "1" else "rows")
        assert bool(eng.roles) == (roles == "1")
        eng.train(rb, 4)
        eng.train_graph(rb, 6, chunk=3)
        eng.check()
        out[roles] = {k: v.clone() for k, v in eng.state_tensors().items()}
        out[roles]["stats"] = eng.stats.clone()
    for k in out["1"]:
        assert torch.equal(out["1"][k], out["0"][k]), k


@pytest.mark.parametrize("layout", ["auto", "rows"])
def test_large_batch_uses_pair_or_row_tile_kernels_and_runs(layout):
    """C3 (B=4096): 256 row tiles do not fit the role split; the pair-tile kernels
    run (C3's default), or with layout "rows" the one-block-per-row-tile kernels
    (stage_path=-1 also refuses the stage path)."""
    eng, rb, c = _engine("c3", "bf16", capacity=20_000, stage_path=-1, layout=layout)
    assert not eng.roles and not eng.wide and eng.pairs == (layout == "auto")
    eng.train_graph(rb, 20, chunk=10)
    eng.check()
    assert all(np.isfinite(eng.losses()))


@pytest.mark.parametrize("cfg,precision,layout", [("c2", "bf16", "auto"), ("c2", "fp32", "roles"),
                                                  ("c3", "bf16", "auto"), ("c3", "fp32", "rows"),
                                                  ("c3_b4001", "fp32", "auto"), ("c3_b4001", "bf16", "auto")])
def test_staged_batch_equals_in_step_gather(cfg, precision, layout):
    """Phase C staging step t+1's batch (sampled and gathered one launch early)
    gives the same bits as phase A gathering it, across graph replays, a replay
    push between calls (the staged record goes stale and phase A gathers), and
    injected indices.  The staged path must actually run.  B = 4001 (ADVICE
    r05): 251 row tiles, so the last pair tile's second tile lies past the
    batch and its LDS rows are zero-filled instead of staged (device RNG)."""
    import ctypes

    import bench
    from sac import _engine as E

    if cfg == "c3_b4001":
        bench.CONFIGS[cfg] = dict(bench.CONFIGS["c3"], batch=4001)
    try:
        _staged_vs_gathered(cfg, precision, layout, ctypes, E)
    finally:
        bench.CONFIGS.pop("c3_b4001", None)


def _staged_vs_gathered(cfg, precision, layout, ctypes, E):
    out = {}
    for stage in ("1", "0"):
        # stage_path=-1 at C3: batch staging is a feature of the row-tile kernels
        eng, rb, c = _engine(cfg, precision, capacity=5000, layout=layout, stage_batch=0 if stage == "1" else -1,
                             stage_path=-1 if cfg.startswith("c3") else 0)
        if cfg == "c3_b4001":
            assert eng.pairs
        eng.train(rb, 3)
        eng.train_graph(rb, 5, chunk=2)
        if stage == "1":
            lib = eng.lib
            lib.sac_engine_debug_staged_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            got = ctypes.c_uint64(0)
            E.check(lib.sac_engine_debug_staged_step(eng.handle, ctypes.byref(got), eng._stream()))
            assert got.value > 0, "phase A never used a staged batch"
        g = np.random.default_rng(5)
        n = 7
        rb.push_batch(g.standard_normal((n, c["obs"]), dtype=np.float32), g.uniform(-1, 1, (n, c["act"])),
                      g.standard_normal(n), g.standard_normal((n, c["obs"]), dtype=np.float32), g.random(n) < 0.1)
        eng.train(rb, 2)
        idx = torch.from_numpy(g.choice(len(rb), size=(2, c["batch"]), replace=True).astype(np.int32))
        eng.train(rb, 2, indices=idx)
        eng.train(rb, 2)
        eng.check()
        out[stage] = {k: v.clone() for k, v in eng.state_tensors().items()}
        out[stage]["stats"] = eng.stats.clone()
    for k in out["1"]:
        assert torch.equal(out["1"][k], out["0"][k]), k


# ---------------------------------------------------------------- hand-off status (round 2)
def test_handoff_timeout_raises_through_the_api(lib):
    """A hand-off spin bound of 0 polls makes every role-split consumer that
    does not find its producer's granules at once give up: the step is invalid,
    the device flag is set, and the Python API (losses(), check(), save_agent)
    raises HandoffTimeout instead of returning the invalid state.  After
    clear_status() and the default bound the engine trains normally again."""
    from sac import _engine as E

    eng, rb, c = _engine("c2", "fp32", capacity=5000)
    assert eng.roles
    eng.train(rb, 2)
    eng.check()
    f = lib.sac_engine_debug_set_spin_limit
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    E.check(f(eng.handle, 0, eng._stream()))
    eng.train(rb, 4)
    with pytest.raises(E.HandoffTimeout):
        eng.losses()
    with pytest.raises(RuntimeError):  # HandoffTimeout is a RuntimeError
        eng.check()
    E.check(f(eng.handle, 1 << 22, eng._stream()))
    eng.clear_status()
    eng.train(rb, 3)
    eng.check()
    assert all(np.isfinite(eng.losses()[:3]))


def test_concurrent_engines_on_streams_match_serial():
    """Two learners on two HIP streams at once (the multi-learner packing that
    contends for CUs) give the same bits as each run alone, and no hand-off
    times out (producer roles sit on the lowest block ids of every launch)."""
    runs = {}
    for mode in ("serial", "concurrent"):
        e1, rb1, _ = _engine("c2", "fp32", seed=1, capacity=5000)
        e2, rb2, _ = _engine("c2", "fp32", seed=2, capacity=5000)
        s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
        torch.cuda.synchronize()
        if mode == "serial":
            with torch.cuda.stream(s1):
                e1.train_graph(rb1, 40, chunk=10)
            s1.synchronize()
            with torch.cuda.stream(s2):
                e2.train_graph(rb2, 40, chunk=10)
            s2.synchronize()
        else:
            for _ in range(4):
                with torch.cuda.stream(s1):
                    e1.train_graph(rb1, 10, chunk=10)
                with torch.cuda.stream(s2):
                    e2.train_graph(rb2, 10, chunk=10)
            torch.cuda.synchronize()
        e1.check()
        e2.check()
        runs[mode] = [{k: v.clone() for k, v in e.state_tensors().items()} for e in (e1, e2)]
    for i in range(2):
        for k in runs["serial"][i]:
            assert torch.equal(runs["serial"][i][k], runs["concurrent"][i][k]), (i, k)


def test_clear_and_refill_invalidates_the_staged_batch():
    """ReplayBuffer.clear() followed by a refill to the same (size, write slot)
    must not let phase A use the batch phase C staged from the old rows: the
    push generation in the replay state differs, so phase A gathers the new
    rows (same bits as a run with staging off)."""
    out = {}
    for stage in ("1", "0"):
        eng, rb, c = _engine("c2", "fp32", capacity=4096, stage_batch=0 if stage == "1" else -1)
        eng.train(rb, 2)  # phase C of step 2 staged step 3's batch from the old rows
        g = np.random.default_rng(9)
        rb.clear()
        n = 4096  # refill to the same size; the write slot wraps back to 0 as before
        rb.push_batch(g.standard_normal((n, c["obs"]), dtype=np.float32), g.uniform(-1, 1, (n, c["act"])),
                      g.standard_normal(n), g.standard_normal((n, c["obs"]), dtype=np.float32), g.random(n) < 0.1)
        assert int(rb.state[0]) == 4096 and int(rb.state[1]) == 0
        eng.train(rb, 2)
        eng.check()
        out[stage] = {k: v.clone() for k, v in eng.state_tensors().items()}
    for k in out["1"]:
        assert torch.equal(out["1"][k], out["0"][k]), k


# ---------------------------------------------------------------- gather kernel (round 2)
@pytest.mark.parametrize("layout", ["records", "soa"])
@pytest.mark.parametrize("obs,act", [(24, 4), (5, 2), (32, 2)])
def test_sample_gather_equals_sampler_plus_gather(lib, obs, act, layout):
    """sac_replay_sample_gather (sampler + row-vectorised gather in one kernel)
    returns the sampler's indices and exactly the rows sac_replay_gather
    returns for them, for 16-B-aligned rows (obs 24/32) and scalar rows (5/2),
    on a wrapped ring."""
    from sac import _engine as E
    from sac.replay_buffer import ReplayBuffer

    cap = 3000
    rb = ReplayBuffer(cap, device=DEV, obs_dim=obs, act_dim=act, layout=layout)
    g = np.random.default_rng(0)
    n = 4100  # wraps: the oldest row sits at slot 1100
    rb.push_batch(g.standard_normal((n, obs), dtype=np.float32), g.uniform(-1, 1, (n, act)).astype(np.float32),
                  g.standard_normal(n), g.standard_normal((n, obs), dtype=np.float32), g.random(n) < 0.1)
    for B in (1, 64, 100, 2999):
        f32 = dict(dtype=torch.float32, device=DEV)
        out = [torch.empty(B, obs, **f32), torch.empty(B, act, **f32), torch.empty(B, **f32),
               torch.empty(B, obs, **f32), torch.empty(B, **f32)]
        idx = torch.empty(B, dtype=torch.int32, device=DEV)
        desc = rb.desc
        E.check(lib.sac_replay_sample_gather(ctypes.byref(desc), B, 5, 17, E.ptr(idx), *[E.ptr(t) for t in out],
                                             E.stream_handle(DEV)))
        ref_idx = torch.empty(B, dtype=torch.int32, device=DEV)
        E.check(lib.sac_replay_sample_indices(ctypes.byref(desc), B, 5, 17, E.ptr(ref_idx), E.stream_handle(DEV)))
        assert torch.equal(idx, ref_idx)
        t = rb.gather(idx.cpu().numpy())
        for a_, b_ in zip(out, t):
            assert torch.equal(a_, b_)
        # and against the host copy of the storage, by ring slot
        li = idx.cpu().numpy().astype(np.int64)
        slot = (int(rb.state[1]) + li) % cap
        assert np.array_equal(out[0].cpu().numpy(), rb.obs.cpu().numpy()[slot])
        assert np.array_equal(out[4].cpu().numpy(), rb.done.cpu().numpy()[slot])


def test_gather_with_replacement_past_capacity(lib):
    """The bandwidth leg of bench.py gathers B = 1,048,576 rows with replacement
    (B > the 1e6-row buffer): the gather is exact at that size too."""
    from sac import _engine as E
    from sac.replay_buffer import ReplayBuffer

    cap, obs, act = 1_000_000, 24, 4
    rb = ReplayBuffer(cap, device=DEV, obs_dim=obs, act_dim=act)
    n = cap + 12_345
    gen = torch.Generator(device=DEV).manual_seed(0)
    rows = torch.randn(n, 2 * obs + act + 2, device=DEV, generator=gen)
    rb.push_batch(rows[:, :obs], rows[:, obs:obs + act], rows[:, obs + act], rows[:, obs + act + 1:2 * obs + act + 1],
                  rows[:, -1] > 0)
    B = 1 << 20
    idx = torch.randint(0, cap, (B,), device=DEV, dtype=torch.int32, generator=gen)
    t = rb.gather(idx)
    slot = (idx.long() + int(rb.state[1])) % cap
    assert torch.equal(t.state, rb.obs[slot]) and torch.equal(t.next_state, rb.next_obs[slot])
    assert torch.equal(t.action, rb.act[slot]) and torch.equal(t.reward, rb.rew[slot])
    assert torch.equal(t.done, rb.done[slot])


def test_c3_full_size_properties():
    """C3 at full size (1e6-row buffer, B = 4096, fp32 parity mode, device
    sampler): 60 graph-replayed steps stay finite with no hand-off timeout, and
    the in-step sampler draws the exported sampler's distinct rows."""
    eng, rb, c = _engine("c3", "fp32")
    assert len(rb) == 1_000_000
    eng.train_graph(rb, 60, chunk=20)
    eng.check()
    losses = eng.losses()
    assert all(np.isfinite(losses)), losses
    assert np.all(np.isfinite(eng.last_targets().cpu().numpy()))
    assert int(eng.rng_step.item()) == 60


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_training_is_layout_independent(precision):
    """The step reads the replay through its field strides: the same rows
    in transition records and in struct-of-arrays give the same bits (device
    sampler, staged next-step batches and graph replay included)."""
    import bench

    out = {}
    for layout in ("records", "soa"):
        eng, rb, c = _engine("c2", precision, capacity=5000)
        if layout == "soa":
            rb = bench.soa_copy(rb)
        assert rb.layout == layout
        eng.train(rb, 3)
        eng.train_graph(rb, 6, chunk=3)
        eng.check()
        out[layout] = {k: v.clone() for k, v in eng.state_tensors().items()}
        out[layout]["stats"] = eng.stats.clone()
    for k in out["records"]:
        assert torch.equal(out["records"][k], out["soa"][k]), k


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_hidden_split_is_used_and_close_to_unsplit(lib, precision):
    """C2 runs the hidden-split role kernels (two workgroups per role and row
    tile); 5 device-sampled steps agree with the unsplit role kernels to
    rounding (the split only changes the summation order of layers 1-2 and of
    layer 0's dW; both paths are checked against the oracle elsewhere)."""
    lib.sac_engine_uses_split.argtypes = [ctypes.c_void_p]
    out = {}
    for split in ("1", "0"):
        eng, rb, c = _engine("c2", precision, capacity=5000, layout="auto" if split == "1" else "roles")
        assert lib.sac_engine_uses_split(eng.handle) == int(split)
        eng.train(rb, 2)
        eng.train_graph(rb, 3, chunk=3)
        eng.check()
        out[split] = {k: v.clone() for k, v in eng.state_tensors().items()}
        out[split]["losses"] = torch.tensor(eng.losses())
    tol = 2e-5 if precision == "fp32" else 2e-3
    for k in out["1"]:
        a, b = out["1"][k].double(), out["0"][k].double()
        assert torch.allclose(a, b, rtol=tol, atol=tol), (k, (a - b).abs().max().item())


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_stage_path_staged_batches_equal_fresh_gathers(precision):
    """The stage path (csrc/sac_wide.h, forced at C3 by stage_path=1) gathers
    step t+1's batch inside step t's last phase-C launch; the first step of
    every call gathers its own.  So one call of 5 steps (device RNG) must equal
    5 calls of one step, bit for bit, and the same with injected indices; graph
    replay equals eager launches."""
    out = {}
    for mode in ("one_call", "per_step", "graph"):
        eng, rb, c = _engine("c3", precision, capacity=12_000, stage_path=1)
        assert eng.wide > 0
        if mode == "one_call":
            eng.train(rb, 5)
        elif mode == "per_step":
            for _ in range(5):
                eng.train(rb, 1)
        else:
            eng.train_graph(rb, 5, chunk=5)
        r9 = np.random.default_rng(9)
        idx = torch.from_numpy(np.stack([r9.choice(len(rb), size=c["batch"], replace=False) for _ in range(3)])
                               .astype(np.int32))
        if mode == "per_step":
            for i in range(3):
                eng.train(rb, 1, indices=idx[i:i + 1])
        else:
            eng.train(rb, 3, indices=idx)
        eng.check()
        out[mode] = {k: v.clone() for k, v in eng.state_tensors().items()}
        out[mode]["stats"] = eng.stats.clone()
    for mode in ("per_step", "graph"):
        for k in out["one_call"]:
            assert torch.equal(out["one_call"][k], out[mode][k]), (mode, k)
