"""CPU ORACLE (test infrastructure only) -- Philox4x32-10 restated in NumPy.

The device panel kernel's throughput mode draws the labour-shock uniform of agent i
in period t from a counter-based Philox4x32-10 generator (Salmon et al., SC'11,
"Parallel random numbers: as easy as 1, 2, 3"; the Random123 reference constants),
SURVEY.md §8d config 2.  This module restates it bit-exactly so tests can pin the
device stream:

    counter = (t, j_lo, j_hi, stream), j = i // 2, key = (seed_lo, seed_hi)
    (x0, x1, x2, x3) = philox4x32_10(counter, key)
    u(2j)     = ((x0 >> 5) * 2**26 + (x1 >> 6)) / 2**53   # in [0, 1), 53 random bits
    u(2j + 1) = ((x2 >> 5) * 2**26 + (x3 >> 6)) / 2**53

(one Philox call serves two agents; every agent still gets its own 53-bit uniform)

(the same 53-bit construction NumPy's MT19937 ``random_sample`` uses).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            if r < 9:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def uniform(t, idx, seed, stream=0):
    """Uniform in [0, 1) for period ``t`` and global agent index ``idx`` (arrays ok)."""
    idx = np.asarray(idx, dtype=np.uint64)
    t = np.asarray(t, dtype=np.uint64)
    seed = int(seed)
    j = idx >> np.uint64(1)
    odd = (idx & np.uint64(1)).astype(bool)
    x0, x1, x2, x3 = philox4x32_10(t.astype(np.uint32) + np.zeros_like(j, dtype=np.uint32),
                                   (j & MASK).astype(np.uint32),
                                   (j >> np.uint64(32)).astype(np.uint32),
                                   np.uint32(stream) + np.zeros_like(j, dtype=np.uint32),
                                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    a = np.where(odd, x2, x0) >> np.uint32(5)
    b = np.where(odd, x3, x1) >> np.uint32(6)
    return (a.astype(np.float64) * 67108864.0 + b.astype(np.float64)) / 9007199254740992.0


def philox_u_source(seed, N, offset=0):
    """u_source for oracle.hark_ks.KSModel: period t of GE iteration g uses counter
    word t' = g * 2**20 + t (stream 0)."""

    def src(ge_iter, t0, t1):
        idx = np.arange(offset, offset + N, dtype=np.uint64)
        return np.stack([uniform(ge_iter * (1 << 20) + t, idx, seed) for t in range(t0, t1)])

    return src
