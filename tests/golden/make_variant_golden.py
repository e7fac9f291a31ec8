"""Generate tests/golden/variants_cover.npz: float64-oracle references (oracle/kymatio_ref.py) of
one random uint8/255 plane for every geometry of tests/variant_geometries.py (the cover of the
reachable kernel variants, tools/variant_cover.py).

Per geometry i (all arrays float32 / int32):
  geoms[i]   (M, N, J, L, max_order)
  {i}_pos    flat spatial positions sampled (all of them when the map holds <= 16 values)
  {i}_ref    (K, npos) the oracle's coefficients at those positions
  {i}_scale  (K,) max |S_ref[k]| over the whole map (the per-coefficient parity denominator)
The input plane is regenerated from `seed_of(geometry)` by the tests (tests/test_gpu_variants.py).

usage: python tests/golden/make_variant_golden.py   (CPU, a fork pool over the host cores; minutes)
"""
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

NSAMPLE = 16


def seed_of(g):
    M, N, J, L, mo = g
    return 1_000_003 * M + 10_007 * N + 101 * J + 7 * L + mo


def plane_of(g):
    M, N = g[0], g[1]
    rng = np.random.default_rng(seed_of(g))
    return (rng.integers(0, 256, (1, M, N), dtype=np.uint8).astype(np.float32) / 255)


def positions_of(g, K, Mo, No):
    n = Mo * No
    if n <= NSAMPLE:
        return np.arange(n, dtype=np.int32)
    rng = np.random.default_rng(seed_of(g) + 1)
    return np.sort(rng.choice(n, NSAMPLE, replace=False)).astype(np.int32)


def one(g):
    from oracle import kymatio_ref as kr
    M, N, J, L, mo = g
    S = kr.Scattering2D(J=J, shape=(M, N), L=L, max_order=mo)(plane_of(g))[0]   # (K, Mo, No)
    K, Mo, No = S.shape
    flat = S.reshape(K, -1)
    pos = positions_of(g, K, Mo, No)
    return (flat[:, pos].astype(np.float32), pos, np.abs(flat).max(axis=1).astype(np.float32))


def main():
    from variant_geometries import COVER
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(one, COVER, chunksize=1)
    arrs = {"geoms": np.array(COVER, np.int32)}
    for i, (ref, pos, scale) in enumerate(res):
        arrs[f"{i}_ref"], arrs[f"{i}_pos"], arrs[f"{i}_scale"] = ref, pos, scale
    out = os.path.join(HERE, "variants_cover.npz")
    np.savez_compressed(out, **arrs)
    print(f"wrote {out}: {len(COVER)} geometries, {os.path.getsize(out) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
