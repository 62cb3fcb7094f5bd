"""CPU restatement of the engine's reparameterisation noise (test infrastructure only: tests/ import it).

The reference draws eps with torch.randn_like (src/Convolutional_VAE.py:162-165, src/Conditional_VAE.py:201-204,
src/Simple_VAE.py:91-93); its values are not a parity contract (any N(0, 1) stream).  The engine draws its own on
the device (csrc/kernels.hip philox_normal4): Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers:
as easy as 1, 2, 3", SC'11; constants of the Random123 reference implementation) keyed by a 64-bit seed, element g
= component g % 4 of the block at counter (g / 4 as 64 bits, 0, 0), Box-Muller on the word pairs.  This restates
both in pure Python / numpy.  Pinned by the Random123 known-answer vectors (tests/test_oracle_cpu.py)."""
from __future__ import annotations

import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32(ctr, key, rounds=10):
    """One Philox4x32 block: ctr 4 x uint32, key 2 x uint32 -> 4 x uint32."""
    c0, c1, c2, c3 = (int(x) & MASK for x in ctr)
    k0, k1 = (int(x) & MASK for x in key)
    for _ in range(rounds):
        p0, p1 = M0 * c0, M1 * c2
        hi0, lo0 = p0 >> 32, p0 & MASK
        hi1, lo1 = p1 >> 32, p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c0, c1, c2, c3


def normals(n, seed, offset=0):
    """Elements offset .. offset + n - 1 of stream `seed` (offset % 4 == 0), float32 Box-Muller as on the device."""
    assert offset % 4 == 0
    out = np.empty(n, np.float32)
    k = np.float32(2.3283064365386963e-10)
    two_pi = np.float32(6.283185307179586)
    for t in range((n + 3) // 4):
        q = offset // 4 + t
        w = philox4x32((q & MASK, q >> 32, 0, 0), (seed & MASK, (seed >> 32) & MASK))
        f = [np.float32(x) for x in w]
        r0 = np.sqrt(np.float32(-2.0) * np.log((f[0] + np.float32(1.0)) * k))
        a0 = two_pi * (f[1] * k)
        r1 = np.sqrt(np.float32(-2.0) * np.log((f[2] + np.float32(1.0)) * k))
        a1 = two_pi * (f[3] * k)
        vals = (r0 * np.cos(a0), r0 * np.sin(a0), r1 * np.cos(a1), r1 * np.sin(a1))
        for j in range(4):
            if 4 * t + j < n:
                out[4 * t + j] = vals[j]
    return out
