"""Oracle for the replay sampler — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module; the product path never does.

Reference semantics (what must hold): ``ReplayBuffer.sample`` draws
``random.sample(self.buffer, batch_size)`` — ``batch_size`` DISTINCT rows,
uniformly, ``ValueError`` when fewer rows are stored
(/root/reference/sac/replay_buffer.py:32-39).  The reference's stream is
CPython's MT19937, which a device sampler cannot reproduce without a host
round trip, so the engine's ``device`` RNG mode uses a different generator
with the same distributional contract, and the ``reference`` RNG mode injects
``random.sample`` indices instead (tests/test_gpu_parity.py).

This file restates that device generator (soft-actor-critic_amd/csrc/
sac_device.h: philox4x32_10, mix32, feistel_make, feistel_perm,
feistel_sample) in plain Python integers, so the host/device exports can be
checked bit-exactly and its properties (distinct, in range, uniform) tested
independently of the C++ code.
"""
from __future__ import annotations

M32 = 0xFFFFFFFF


def philox4x32_10(c, k0, k1):
    """Philox4x32 with 10 rounds (Salmon et al. 2011); c: 4 uint32 counters."""
    c = list(c)
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        n0 = ((p1 >> 32) ^ c[1] ^ k0) & M32
        n2 = ((p0 >> 32) ^ c[3] ^ k1) & M32
        c[1] = p1 & M32
        c[3] = p0 & M32
        c[0], c[2] = n0, n2
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c


def mix32(x):
    """lowbias32 integer hash."""
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


class Feistel:
    """6-round balanced Feistel permutation of [0, 2^bits), keys from Philox(seed, step)."""

    def __init__(self, seed: int, step: int, size: int):
        bits = 2
        while bits < 62 and (1 << bits) < size:
            bits += 1
        if bits & 1:
            bits += 1
        self.half = bits // 2
        self.mask = M32 if self.half >= 32 else (1 << self.half) - 1
        s0, s1 = seed & M32, (seed >> 32) & M32
        lo, hi = step & M32, (step >> 32) & M32
        c = philox4x32_10([lo, hi, M32, 0x5A3F0001], s0, s1)
        d = philox4x32_10([lo, hi, M32, 0x5A3F0002], s0, s1)
        self.key = c + d[:2]

    def perm(self, x: int) -> int:
        L, R = (x >> self.half) & self.mask, x & self.mask
        for k in self.key:
            L, R = R, L ^ (mix32(R ^ k) & self.mask)
        return (L << self.half) | R

    def sample(self, b: int, size: int) -> int:
        """b-th element of the permutation restricted to [0, size) (cycle walking)."""
        y = self.perm(b)
        it = 0
        while y >= size and it < 4096:
            y = self.perm(y)
            it += 1
        return y


def sample_indices(size: int, batch: int, seed: int, step: int):
    """Logical replay positions (0 = oldest) of one device-sampled minibatch."""
    if batch > size:
        raise ValueError(f"Not enough samples in the replay buffer to sample {batch} transitions. "
                         f"Current size: {size}")
    f = Feistel(seed, step, size)
    return [f.sample(b, size) for b in range(batch)]


# ----------------------------------------------------------------------------- eps
# The reference draws each rsample's eps from torch's generator
# (/root/reference/sac/models.py:79-87 -> torch/distributions/normal.py:83-86,
# one [B, act] draw for the target (agent.py:204) and one for the actor
# (agent.py:241)).  The engine's device RNG mode draws them instead from
# Philox4x32-10 + Box-Muller (sac_device.h philox_normal2): for row b, draw
# `which` (0 target, 1 actor) and pair p, counter = (step lo, step hi, b,
# which << 16 | p), key = (seed lo, seed hi); u1 = (c0 >> 8) + 1 over 2^24 in
# (0, 1], u2 = (c1 >> 8) / 2^24 in [0, 1); r = sqrt(-2 log u1);
# eps[b][2p] = r cos(2 pi u2), eps[b][2p + 1] = r sin(2 pi u2), all in fp32.
# Vectorised over (which, b, p) with uint64 lanes; the float32 log / sqrt / sin
# / cos are numpy's, so a value may differ from the device's by an ulp or two.

def _philox_np(c0, c1, c2, c3, k0, k1):
    import numpy as np

    m = np.uint64(M32)
    c = [np.asarray(x, np.uint64) & m for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0 & M32), np.uint64(k1 & M32)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]  # < 2^64: exact in uint64
        p1 = np.uint64(0xCD9E8D57) * c[2]
        n0 = ((p1 >> np.uint64(32)) ^ c[1] ^ k0) & m
        n2 = ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & m
        c[1] = p1 & m
        c[3] = p0 & m
        c[0], c[2] = n0, n2
        k0 = (k0 + np.uint64(0x9E3779B9)) & m
        k1 = (k1 + np.uint64(0xBB67AE85)) & m
    return c


def eps_draws(seed: int, step: int, batch: int, act_dim: int):
    """[2][batch][act_dim] float32: the target (0) and actor (1) eps of device
    RNG step ``step`` (what sac_debug_eps_host / the fused step compute)."""
    import numpy as np

    NP = (act_dim + 1) // 2
    which, b, p = np.meshgrid(np.arange(2, dtype=np.uint64), np.arange(batch, dtype=np.uint64),
                              np.arange(NP, dtype=np.uint64), indexing="ij")
    c = _philox_np(np.full(which.shape, step & M32, np.uint64), np.full(which.shape, (step >> 32) & M32, np.uint64),
                   b, (which << np.uint64(16)) | p, seed & M32, (seed >> 32) & M32)
    scale = np.float32(5.9604644775390625e-8)  # 2^-24
    u1 = ((c[0] >> np.uint64(8)) + np.uint64(1)).astype(np.float32) * scale
    u2 = (c[1] >> np.uint64(8)).astype(np.float32) * scale
    r = np.sqrt(np.float32(-2.0) * np.log(u1))
    ang = np.float32(6.283185307179586) * u2
    n0, n1 = r * np.cos(ang), r * np.sin(ang)
    out = np.empty((2, batch, 2 * NP), np.float32)
    out[..., 0::2] = n0
    out[..., 1::2] = n1
    return out[..., :act_dim].copy()
