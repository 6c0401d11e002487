"""NumPy mirror of the device Philox4x32-10 RNG (csrc/include/cgnn_common.h).

The integer part is bit-identical to the HIP implementation, so the CPU path
and the GPU path draw the *same* noise for the same (key, counter); only the
final float transcendental (log / cos) may differ by an ulp.  This is what
makes GPU results reproducible on CPU and independent of the number of GPUs
(SURVEY §2.6 B14, §7.4 item 4).
"""
from __future__ import annotations

import hashlib

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

RNG_NODE_NOISE = 1
RNG_CONF_NOISE = 2
RNG_PARAM_INIT = 3
RNG_RFF_FREQ = 4
RNG_DROPOUT = 5
RNG_SAMPLE = 6


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; all inputs broadcastable uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(int(k0) & 0xFFFFFFFF)
    k1 = np.uint64(int(k1) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c1 ^ k0
        n1 = lo1
        n2 = hi0 ^ c3 ^ k1
        n3 = lo0
        c0, c1, c2, c3 = n0, n1, n2, n3
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def u01(x):
    """24-bit uniform in (0,1), centred in its bucket (matches ``u01`` on device)."""
    x = np.asarray(x, dtype=np.uint32)
    return ((x >> np.uint32(8)).astype(np.float64) + 0.5) * (1.0 / 16777216.0)


def normal(k0, k1, a, b, step, purpose, dtype=np.float32):
    """Standard normals for counters (a, b, step, purpose), Box-Muller cos branch."""
    r0, r1, _, _ = philox4x32_10(a, b, step, purpose, k0, k1)
    u1 = u01(r0)
    u2 = u01(r1)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return z.astype(dtype)


def uniform(k0, k1, a, b, step, purpose, word=2, dtype=np.float32):
    r = philox4x32_10(a, b, step, purpose, k0, k1)
    return u01(r[word]).astype(dtype)


def model_key(seed: int, *salt) -> tuple:
    """64-bit Philox key for one model, a pure function of (seed, salt...)."""
    h = hashlib.blake2b(repr((int(seed),) + tuple(salt)).encode(), digest_size=8).digest()
    v = int.from_bytes(h, "little")
    return v & 0xFFFFFFFF, (v >> 32) & 0xFFFFFFFF


def numpy_rng(seed: int, *salt) -> np.random.Generator:
    """Host-side generator for non-hot randomness (subsampling, search moves)."""
    h = hashlib.blake2b(repr(("np", int(seed)) + tuple(salt)).encode(), digest_size=8).digest()
    return np.random.default_rng(int.from_bytes(h, "little"))
