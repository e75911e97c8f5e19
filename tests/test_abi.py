"""The C-ABI boundary (include/*.h) without a GPU: the library loads, exports
every declared symbol, the ctypes mirror has the C layouts, and the host-only
entry points (validation, workspace planning, names, host sampler) behave."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

INCLUDE = os.path.join(ROOT, "include")


def declared_functions(header):
    text = open(os.path.join(INCLUDE, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(sac_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    from sac import _engine as E

    if not os.path.exists(E.library_path()):
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True)
    return E.load_library()


def test_header_parse_sane():
    fns = declared_functions("sac_engine.h")
    assert "sac_engine_train" in fns and "sac_replay_gather" in fns and len(fns) >= 14


@pytest.mark.parametrize("header", ["sac_engine.h", "sac_engine_testing.h"])
def test_library_exports_every_declared_symbol(lib, header):
    missing = [f for f in declared_functions(header) if not hasattr(lib, f)]
    assert not missing, f"{header}: not exported by libsac_engine.so: {missing}"


def test_ctypes_signatures_cover_boundary():
    from sac import _engine as E

    assert sorted(E.SIGNATURES) == declared_functions("sac_engine.h")


def _c_layout(tmp_path):
    """sizeof/offsetof of the boundary structs as the C compiler lays them out."""
    fields = {
        "sac_engine_config": ["obs_dim", "act_dim", "batch", "q_layers", "q_dims", "q_hidden_act", "q_out_act",
                              "pi_layers", "pi_dims", "pi_hidden_act", "pi_out_act", "gamma", "tau", "log_std_min",
                              "log_std_max", "action_scale", "actor_lr", "critic_lr", "alpha_lr", "beta1", "beta2",
                              "adam_eps", "auto_entropy", "target_entropy", "precision", "seed", "layout",
                              "stage_path", "stage_batch", "upd_parts", "upd_threads"],
        "sac_engine_buffers": ["pi", "q1", "q2", "q1t", "q2t", "pi_m", "pi_v", "q1_m", "q1_v", "q2_m", "q2_v",
                               "alpha_state", "opt_steps", "rng_step", "stats", "workspace", "workspace_bytes"],
        "sac_replay": ["obs", "act", "rew", "next_obs", "done", "capacity", "obs_dim", "act_dim", "state",
                       "row_stride"],
    }
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "sac_engine.h"', "int main(void) {"]
    for st, fs in fields.items():
        src.append(f'printf("{st} size %zu\\n", sizeof({st}));')
        for f in fs:
            src.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", INCLUDE, str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    lay = {}
    for line in out.splitlines():
        st, f, v = line.split()
        lay[(st, f)] = int(v)
    return lay


def test_ctypes_struct_layouts_match_c(tmp_path):
    from sac import _engine as E

    lay = _c_layout(tmp_path)
    for st, cls in (("sac_engine_config", E.EngineConfig), ("sac_engine_buffers", E.EngineBuffers),
                    ("sac_replay", E.ReplayDesc)):
        assert ctypes.sizeof(cls) == lay[(st, "size")], st
        for name, _ in cls._fields_:
            assert getattr(cls, name).offset == lay[(st, name)], (st, name)


def _config(E, obs=24, act=4, hidden=(256, 256), batch=256, precision=1):
    c = E.EngineConfig()
    c.obs_dim, c.act_dim, c.batch = obs, act, batch
    qd = [obs + act, *hidden, 1]
    pd = [obs, *hidden, 2 * act]
    c.q_layers, c.pi_layers = len(qd) - 1, len(pd) - 1
    for i, d in enumerate(qd):
        c.q_dims[i] = d
    for i, d in enumerate(pd):
        c.pi_dims[i] = d
    c.q_hidden_act = c.pi_hidden_act = 1
    c.gamma, c.tau, c.log_std_min, c.log_std_max, c.action_scale = 0.99, 0.005, -20.0, 2.0, 1.0
    c.actor_lr = c.critic_lr = c.alpha_lr = 3e-4
    c.beta1, c.beta2, c.adam_eps = 0.9, 0.999, 1e-8
    c.auto_entropy, c.target_entropy, c.precision = 1, -float(act), precision
    return c


def test_workspace_planning_and_validation(lib):
    from sac import _engine as E

    c2 = _config(E)
    ws = lib.sac_engine_workspace_bytes(ctypes.byref(c2))
    assert ws > 0
    c3 = _config(E, batch=4096)
    assert lib.sac_engine_workspace_bytes(ctypes.byref(c3)) > ws  # per-row stashes grow with the batch
    bad = _config(E)
    bad.q_dims[0] = 27  # must be obs + act
    assert lib.sac_engine_workspace_bytes(ctypes.byref(bad)) == 0
    bad = _config(E, batch=0)
    assert lib.sac_engine_workspace_bytes(ctypes.byref(bad)) == 0
    bad = _config(E)
    bad.pi_dims[bad.pi_layers] = 5  # policy head must be 2 * act
    assert lib.sac_engine_workspace_bytes(ctypes.byref(bad)) == 0


def test_names_and_version(lib):
    assert lib.sac_version().decode()
    names = [lib.sac_phase_kernel_name(i).decode() for i in range(4)]
    assert names == ["sac_target_critic", "sac_critic_update", "sac_actor", "sac_actor_update"]
    assert lib.sac_phase_kernel_name(9).decode() == ""


def test_create_rejects_null_and_reports_error(lib):
    from sac import _engine as E

    out = ctypes.c_void_p()
    rc = lib.sac_engine_create(None, None, None, ctypes.byref(out))
    assert rc == -1 and lib.sac_last_error().decode()
    with pytest.raises(E.EngineError):
        E.check(rc)


def _host_sample(lib, size, batch, seed, step):
    f = lib.sac_debug_sample_indices_host
    f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    out = np.zeros(batch, np.int32)
    assert f(size, batch, seed, step, out.ctypes.data) == 0
    return out


@pytest.mark.parametrize("size,batch", [(1, 1), (7, 7), (100, 64), (1000, 256), (1_000_000, 256), (65_537, 4096)])
def test_host_sampler_matches_oracle(lib, size, batch):
    from oracle import sampler_oracle as S

    for step in (0, 1, 12345):
        got = _host_sample(lib, size, batch, 7, step)
        want = S.sample_indices(size, batch, 7, step) if batch <= 512 else None
        if want is not None:
            assert got.tolist() == want
        assert len(set(got.tolist())) == batch  # distinct, like random.sample
        assert got.min() >= 0 and got.max() < size


def test_host_sampler_rejects_oversized_batch(lib):
    f = lib.sac_debug_sample_indices_host
    f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    out = np.zeros(8, np.int32)
    assert f(4, 8, 0, 0, out.ctypes.data) == -1


def test_host_sampler_is_uniform(lib):
    """Marginal of each slot over many steps is uniform (chi-square), and the
    steps are independent draws (different subsets)."""
    size, batch, steps = 200, 50, 2000
    counts = np.zeros(size)
    first = np.zeros(size)
    seen = set()
    for t in range(steps):
        idx = _host_sample(lib, size, batch, 3, t)
        counts[idx] += 1
        first[idx[0]] += 1
        seen.add(tuple(sorted(idx.tolist())))
    exp = steps * batch / size
    chi = ((counts - exp) ** 2 / exp).sum()
    assert chi < size + 5 * np.sqrt(2 * size), chi  # dof = size - 1
    exp1 = steps / size
    chi1 = ((first - exp1) ** 2 / exp1).sum()
    assert chi1 < size + 5 * np.sqrt(2 * size), chi1
    assert len(seen) == steps


@pytest.mark.parametrize("seed,step,B,A", [(0, 0, 256, 4), (7, 12345, 1000, 3), (2**40 + 5, 2**33 + 1, 64, 1),
                                           (3, 17, 4096, 2)])
def test_host_eps_matches_oracle(lib, seed, step, B, A):
    """The device RNG's eps (sac_debug_eps_host: the fused step's inline
    philox_normal2 compiled for the host) against oracle/sampler_oracle.py's
    independent numpy restatement: the same Philox words and fp32 Box-Muller,
    so equal up to the libm / numpy float32 log, sin, cos (2 ulps)."""
    from oracle import sampler_oracle as S

    f = lib.sac_debug_eps_host
    f.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    out = np.zeros((2, B, A), np.float32)
    assert f(seed, step, B, A, out.ctypes.data) == 0
    want = S.eps_draws(seed, step, B, A)
    np.testing.assert_allclose(out, want, rtol=1e-6, atol=1e-6)
    assert np.mean(out == want) > 0.5
    assert f(seed, step, 0, A, out.ctypes.data) == -1  # empty batch rejected
