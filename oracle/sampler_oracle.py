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
