"""The PyTorch custom-op boundary (torch.ops.sac_hip, csrc/sac_torch_ops.cpp).

CPU: the op library loads, registers every op SURVEY §8(b) names with the
declared mutation annotations, and its Meta kernels give the output shapes.
GPU (-m gpu): the ops are bit-identical to the ctypes C-ABI calls they wrap,
run on the current stream, and capture under torch.cuda.graph."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import PKG

OPS = ("bind_engine_library", "replay_push", "replay_gather", "replay_sample", "replay_sample_gather", "train_step", "train_graph",
       "policy_act")


@pytest.fixture(scope="module")
def ops():
    from sac import _engine as E

    if not (os.path.exists(E.library_path()) and os.path.exists(E.ops_library_path())):
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True)
    return E.ops()


def test_every_op_registered_with_mutation_annotations(ops):
    for name in OPS:
        assert hasattr(ops, name), name
    schema = {name: str(getattr(ops, name).default._schema) for name in OPS}
    assert "Tensor(a!) storage" in schema["replay_push"] and "Tensor(b!) state" in schema["replay_push"]
    assert "Tensor(a!)[] state" in schema["train_step"] and "Tensor(a!)[] state" in schema["train_graph"]
    assert "Tensor? indices=None" in schema["train_step"]
    for name in ("replay_gather", "replay_sample", "replay_sample_gather", "policy_act"):
        assert "!" not in schema[name], name  # read-only inputs, fresh outputs


def test_meta_kernels_give_shapes(ops):
    cap, O, A = 100, 24, 4
    stride = 64
    storage = torch.empty(cap * stride, device="meta")
    state = torch.empty(3, dtype=torch.int64, device="meta")
    layout = [cap, O, A, stride, 0, 2 * O, 2 * O + A, O, 2 * O + A + 1]
    idx = torch.empty(37, dtype=torch.int32, device="meta")
    s, a, r, s2, d = ops.replay_gather(storage, state, layout, idx)
    assert [tuple(x.shape) for x in (s, a, r, s2, d)] == [(37, O), (37, A), (37,), (37, O), (37,)]
    out = ops.replay_sample_gather(storage, state, layout, 16, 0, 0)
    assert out[0].dtype == torch.int32 and tuple(out[0].shape) == (16,) and tuple(out[1].shape) == (16, O)
    assert tuple(ops.replay_sample(storage, state, layout, 8, 0, 0).shape) == (8,)
    obs = torch.empty(5, O, device="meta")
    act, lp = ops.policy_act(1, obs, None, A, False)
    assert tuple(act.shape) == (5, A) and lp.numel() == 0
    act, lp = ops.policy_act(1, obs, torch.empty(5, A, device="meta"), A, True)
    assert tuple(lp.shape) == (5,)


def test_ops_reject_cpu_tensors(ops):
    storage = torch.zeros(100 * 16)
    state = torch.zeros(3, dtype=torch.int64)
    with pytest.raises(NotImplementedError, match="CPU"):  # CUDA and Meta kernels only: no CPU fallback
        ops.replay_gather(storage, state, [100, 3, 1, 16, 0, 6, 7, 3, 8], torch.zeros(4, dtype=torch.int32))


# ---------------------------------------------------------------- GPU
DEV = torch.device("cuda", 0)


def _engine(precision="fp32", seed=0, capacity=4096):
    import bench

    c = dict(bench.CONFIGS["c2"])
    bench.CONFIGS["c2"] = dict(c, capacity=capacity)
    try:
        return bench.build_engine("c2", precision, seed, DEV)
    finally:
        bench.CONFIGS["c2"] = c


def _state_equal(e1, e2):
    s1, s2 = e1.state_tensors(), e2.state_tensors()
    for k in s1:
        assert torch.equal(s1[k], s2[k]), k
    assert torch.equal(e1.stats, e2.stats)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_train_step_op_equals_ctypes_abi(ops, precision):
    """torch.ops.sac_hip.train_step == sac_engine_train through ctypes, bit for
    bit, with injected indices/eps (2 steps) and then with the device sampler."""
    from sac import _engine as E

    (e1, rb1, c), (e2, rb2, _) = _engine(precision), _engine(precision)
    B, A = c["batch"], c["act"]
    g = np.random.default_rng(5)
    idx = torch.from_numpy(g.choice(len(rb1), size=(2, B), replace=False).astype(np.int32)).to(DEV)
    eps = torch.from_numpy(g.standard_normal((2, 2, B, A)).astype(np.float32)).to(DEV)
    lib = E.load_library()
    E.check(lib.sac_engine_train(e1.handle, ctypes.byref(rb1.desc), 2, E.ptr(idx), E.ptr(eps), E.stream_handle(DEV)))
    ops.train_step(e2.handle.value, e2.state_list, rb2.storage, rb2.state, rb2.layout_spec, 2, idx, eps)
    torch.cuda.synchronize()
    _state_equal(e1, e2)
    E.check(lib.sac_engine_train(e1.handle, ctypes.byref(rb1.desc), 3, None, None, E.stream_handle(DEV)))
    ops.train_step(e2.handle.value, e2.state_list, rb2.storage, rb2.state, rb2.layout_spec, 3)
    torch.cuda.synchronize()
    _state_equal(e1, e2)
    e1.check()
    e2.check()


@pytest.mark.gpu
def test_train_step_op_captures_under_torch_cuda_graph(ops):
    """The op is capturable by torch.cuda.graph on a side stream (no host
    sync, no allocation): replaying the captured step 4 times == 4 eager steps
    (device sampler; its RNG step lives in device memory)."""
    (e1, rb1, _), (e2, rb2, _) = _engine("fp32"), _engine("fp32")
    for _ in range(4):
        ops.train_step(e1.handle.value, e1.state_list, rb1.storage, rb1.state, rb1.layout_spec, 1)
    torch.cuda.synchronize()
    snap = e2.snapshot()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.train_step(e2.handle.value, e2.state_list, rb2.storage, rb2.state, rb2.layout_spec, 1)
    torch.cuda.synchronize()
    e2.restore(snap)  # capture does not run the step; restore anyway in case a backend executes it
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    _state_equal(e1, e2)
    e2.check()


@pytest.mark.gpu
def test_replay_ops_equal_ctypes_abi(ops):
    """replay_gather / replay_sample / replay_sample_gather ops == the ctypes
    entry points on the same replay (records and struct-of-arrays layouts)."""
    from sac import _engine as E
    from sac.replay_buffer import ReplayBuffer

    lib = E.load_library()
    for layout in ("records", "soa"):
        rb = ReplayBuffer(1000, device=DEV, obs_dim=24, act_dim=4, layout=layout)
        g = np.random.default_rng(1)
        n = 900
        rb.push_batch(g.standard_normal((n, 24), dtype=np.float32), g.standard_normal((n, 4), dtype=np.float32),
                      g.standard_normal(n, dtype=np.float32), g.standard_normal((n, 24), dtype=np.float32),
                      g.random(n) < 0.2)
        idx = torch.from_numpy(g.integers(0, n, 300).astype(np.int32)).to(DEV)
        got = ops.replay_gather(rb.storage, rb.state, rb.layout_spec, idx)
        f = dict(dtype=torch.float32, device=DEV)
        want = [torch.empty(300, 24, **f), torch.empty(300, 4, **f), torch.empty(300, **f), torch.empty(300, 24, **f),
                torch.empty(300, **f)]
        E.check(lib.sac_replay_gather(ctypes.byref(rb.desc), E.ptr(idx), 300, *[E.ptr(t) for t in want],
                                      E.stream_handle(DEV)))
        torch.cuda.synchronize()
        for a, b in zip(got, want):
            assert torch.equal(a, b), layout
        sidx = ops.replay_sample(rb.storage, rb.state, rb.layout_spec, 256, 9, 4)
        ref = torch.empty(256, dtype=torch.int32, device=DEV)
        E.check(lib.sac_replay_sample_indices(ctypes.byref(rb.desc), 256, 9, 4, E.ptr(ref), E.stream_handle(DEV)))
        torch.cuda.synchronize()
        assert torch.equal(sidx, ref)
        gidx, *rows = ops.replay_sample_gather(rb.storage, rb.state, rb.layout_spec, 256, 9, 4)
        assert torch.equal(gidx, ref)
        for a, b in zip(rows, ops.replay_gather(rb.storage, rb.state, rb.layout_spec, ref)):
            assert torch.equal(a, b), layout


@pytest.mark.gpu
def test_policy_act_op_on_current_stream(ops):
    """policy_act runs on torch's current stream: launched on a side stream and
    waited for, it equals the default-stream result."""
    eng, _, c = _engine("fp32")
    g = np.random.default_rng(2)
    obs = torch.from_numpy(g.standard_normal((64, c["obs"]), dtype=np.float32)).to(DEV)
    eps = torch.from_numpy(g.standard_normal((64, c["act"]), dtype=np.float32)).to(DEV)
    a0, lp0 = ops.policy_act(eng.handle.value, obs, eps, c["act"], True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        a1, lp1 = ops.policy_act(eng.handle.value, obs, eps, c["act"], True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(a0, a1) and torch.equal(lp0, lp1)
    det, none = ops.policy_act(eng.handle.value, obs, None, c["act"], True)
    assert none.numel() == 0 and det.shape == (64, c["act"])
