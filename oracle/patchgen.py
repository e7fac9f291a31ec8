"""Host restatement of ``wst_patch_generate`` (include/wst_hip.h) -- TEST INFRASTRUCTURE ONLY.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11: multipliers 0xD2511F53 / 0xCD9E8D57, Weyl
key increments 0x9E3779B9 / 0xBB67AE85, 10 rounds) in vectorised numpy, so the c3 tests can
recreate any patch by its global index and hand it to the kymatio oracle.  Only tests/ and
bench.py's checker import it.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(c, np.uint32) for c in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = c0.astype(np.uint64) * M0
            p1 = c2.astype(np.uint64) * M1
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def generate_patches_u8(seed: int, first: int, n: int, C: int, H: int, W: int) -> np.ndarray:
    """uint8 (n, C, H, W): element e of patch p = byte e & 15 of Philox(counter (e >> 4, 0, p,
    p >> 32), key (seed, (seed >> 32) ^ 0x3C6EF372))."""
    per = C * H * W
    nblk = (per + 15) // 16
    q = np.arange(nblk, dtype=np.uint64)
    out = np.empty((n, nblk * 16), np.uint8)
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32(((seed >> 32) & 0xFFFFFFFF) ^ 0x3C6EF372)
    for i in range(n):
        p = first + i
        w = philox4x32_10(q & MASK, q >> np.uint64(32), np.full(nblk, p & 0xFFFFFFFF, np.uint64),
                          np.full(nblk, p >> 32, np.uint64), k0, k1)
        words = np.stack(w, axis=1).astype("<u4")          # (nblk, 4) little-endian words
        out[i] = words.view(np.uint8).reshape(-1)
    return out[:, :per].reshape(n, C, H, W)
