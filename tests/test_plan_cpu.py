"""The engine's launch plan on the CPU (no GPU needed): sac_engine_create runs
the whole planner -- phase layouts, update tiles with their batch parts and
bias blocks, the stage path's job list -- before its first HIP call.  On a
machine without a GPU it must therefore stop at that first HIP call
(SAC_E_HIP), never at the planner's own consistency check ("internal: ...",
SAC_E_INVALID): a mismatch between the tiles the planner counts (the grids of
phases B and D) and the tiles it builds would make the update kernels read
descriptors that do not exist.  Every bench config, both precisions, and the
diagnostic layouts sac_engine_config's override fields select (the library
reads no environment: tested on its dynamic symbol table)."""
import ctypes
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "soft-actor-critic_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from sac import _engine as E  # noqa: E402

SAC_E_INVALID, SAC_E_HIP = -1, -2


def _cfg(name, precision):
    c = bench.CONFIGS[name]
    cfg = E.EngineConfig()
    cfg.obs_dim, cfg.act_dim, cfg.batch = c["obs"], c["act"], c["batch"]
    qd = [c["obs"] + c["act"]] + c["hidden"] + [1]
    pd = [c["obs"]] + c["hidden"] + [2 * c["act"]]
    cfg.q_layers, cfg.pi_layers = len(qd) - 1, len(pd) - 1
    for i, d in enumerate(qd):
        cfg.q_dims[i] = d
    for i, d in enumerate(pd):
        cfg.pi_dims[i] = d
    cfg.q_hidden_act = cfg.pi_hidden_act = 1  # relu
    cfg.q_out_act = cfg.pi_out_act = 0
    cfg.gamma, cfg.tau = 0.99, 0.005
    cfg.log_std_min, cfg.log_std_max, cfg.action_scale = -20.0, 2.0, 1.0
    cfg.actor_lr = cfg.critic_lr = cfg.alpha_lr = 3e-4
    cfg.beta1, cfg.beta2, cfg.adam_eps = 0.9, 0.999, 1e-8
    cfg.auto_entropy, cfg.target_entropy = 1, -float(c["act"])
    cfg.precision = E.PREC_FP32 if precision == "fp32" else E.PREC_BF16
    cfg.seed = 0
    return cfg


@pytest.mark.parametrize("override", ["", "stage_batch=-1", "layout=1", "layout=2", "layout=3",
                                      "layout=3,upd_threads=512", "upd_parts=4", "upd_threads=1024",
                                      "stage_path=1", "stage_path=-1"])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", sorted(bench.CONFIGS))
def test_plan_is_consistent(name, precision, override):
    lib = E.load_library()
    cfg = _cfg(name, precision)
    for kv in filter(None, override.split(",")):
        k, v = kv.split("=")
        setattr(cfg, k, int(v))
    ws = lib.sac_engine_workspace_bytes(ctypes.byref(cfg))
    assert ws > 0, lib.sac_last_error()
    bufs = E.EngineBuffers(*([0x1000] * 15), 0x100000, ws)  # never dereferenced before the first HIP call
    out = ctypes.c_void_p()
    rc = lib.sac_engine_create(ctypes.byref(cfg), ctypes.byref(bufs), None, ctypes.byref(out))
    msg = lib.sac_last_error().decode()
    if rc == 0:  # a GPU is present: the engine exists; destroy it
        lib.sac_engine_destroy(out)
        pytest.skip("GPU present: the planner ran for real")
    assert "internal" not in msg, msg
    if cfg.layout and rc == SAC_E_INVALID:  # an explicit layout the shape cannot take fails, never falls back
        assert "layout override cannot be honoured" in msg, msg
        assert (name, cfg.layout) in HONOUR_REFUSED, (name, cfg.layout, msg)
        return
    assert (name, cfg.layout) not in HONOUR_REFUSED, (name, cfg.layout)
    assert rc == SAC_E_HIP, (rc, msg)


# (config, forced layout) pairs the planner cannot honour: the per-network role
# kernels need 6 workgroups per row tile co-resident (C3: 256 row tiles); the
# row and pair tiles hold 2R rows of every layer, which at obs 216 (C4') does
# not fit the CU's LDS (that config runs the role kernels by default)
HONOUR_REFUSED = {("c3", 1), ("c4w", 2), ("c4w", 3)}


def test_unhonourable_layout_override_fails():
    """layout=roles at C3 (1536 role workgroups > 256 CUs) used to
    fall back silently to other kernels; it now fails in create with
    SAC_E_INVALID, before any HIP call, like stage_path = -1 on a shape that
    needs the stage path."""
    lib = E.load_library()
    cfg = _cfg("c3", "fp32")
    cfg.layout = 1
    ws = lib.sac_engine_workspace_bytes(ctypes.byref(cfg))
    bufs = E.EngineBuffers(*([0x1000] * 15), 0x100000, ws)
    out = ctypes.c_void_p()
    rc = lib.sac_engine_create(ctypes.byref(cfg), ctypes.byref(bufs), None, ctypes.byref(out))
    if rc == 0:
        lib.sac_engine_destroy(out)
        pytest.fail("layout=roles honoured at C3")
    assert rc == SAC_E_INVALID and "cannot be honoured: roles" in lib.sac_last_error().decode()


def _create_rc(obs, act, hidden, batch=64):
    bench.CONFIGS["_wide"] = dict(obs=obs, act=act, hidden=hidden, batch=batch, capacity=256)
    try:
        cfg = _cfg("_wide", "fp32")
    finally:
        del bench.CONFIGS["_wide"]
    lib = E.load_library()
    ws = lib.sac_engine_workspace_bytes(ctypes.byref(cfg))
    bufs = E.EngineBuffers(*([0x1000] * 15), 0x100000, ws)
    out = ctypes.c_void_p()
    rc = lib.sac_engine_create(ctypes.byref(cfg), ctypes.byref(bufs), None, ctypes.byref(out))
    if rc == 0:
        lib.sac_engine_destroy(out)
        pytest.skip("GPU present: the planner ran for real")
    return rc, lib.sac_last_error().decode()


@pytest.mark.parametrize("obs,act,hidden", [(300, 6, [256, 256]), (24, 4, [512, 512]), (24, 4, [384, 384]),
                                            (17, 6, [400, 300]), (24, 4, [1024, 1024, 512])])
def test_shapes_past_the_lds_layout_take_the_stage_path(obs, act, hidden):
    """Widths whose phase-kernel workgroup would need more than the CU's 160 KiB
    of LDS (hidden layers past 256, inputs past 256 with [256, 256] nets) are
    planned on the layer-synchronous stage path (csrc/sac_wide.h), which takes
    any width: the planner succeeds and creation stops at its first HIP call."""
    rc, msg = _create_rc(obs, act, hidden)
    assert "internal" not in msg, msg
    assert rc == SAC_E_HIP, (rc, msg)


def test_one_wide_hidden_layer_is_refused():
    """A single hidden layer too wide for the phase kernels' LDS (the stage path
    needs two hidden layers) fails in sac_engine_create with SAC_E_INVALID and
    the byte count, before any HIP call."""
    rc, msg = _create_rc(24, 4, [1024])
    assert rc == SAC_E_INVALID and "B of LDS per workgroup (max 163840)" in msg, (rc, msg)


@pytest.mark.parametrize("field,value", [("layout", 4), ("stage_path", 2), ("stage_batch", 1), ("upd_parts", 5),
                                         ("upd_threads", 256)])
def test_bad_layout_override_is_refused(field, value):
    """Out-of-range override fields fail validation (SAC_E_INVALID) in both the
    workspace query and create, before any HIP call."""
    lib = E.load_library()
    cfg = _cfg("c2", "fp32")
    setattr(cfg, field, value)
    assert lib.sac_engine_workspace_bytes(ctypes.byref(cfg)) == 0
    bufs = E.EngineBuffers(*([0x1000] * 15), 0x100000, 1 << 30)
    out = ctypes.c_void_p()
    rc = lib.sac_engine_create(ctypes.byref(cfg), ctypes.byref(bufs), None, ctypes.byref(out))
    assert rc == SAC_E_INVALID and "layout override" in lib.sac_last_error().decode()


def test_engine_library_reads_no_environment():
    """the product library takes every layout choice from
    sac_engine_config; no getenv / secure_getenv import in its dynamic symbols
    (the SAC_STAMPS diagnostic build may read one)."""
    import subprocess

    syms = subprocess.run(["nm", "-D", "--undefined-only", E.library_path()], capture_output=True, text=True,
                          check=True).stdout
    assert "getenv" not in syms, [ln for ln in syms.splitlines() if "getenv" in ln]
