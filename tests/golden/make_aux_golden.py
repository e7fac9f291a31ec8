"""Golden fixtures of the operators either side of the WST path (rows F2, F4), generated from
oracle/reference_ops.py (the reference's own formulas and numpy/scipy calls).

* noise_<type>.npz: two 32x32x3 uint8 images (seed 0), the draws add_noise.py makes
  (np.random.seed(100 + type index), numpy's legacy global RNG) and the reference's output.
* advstats.npz: uint8 planes (several geometries, random + tie-heavy structured content), the
  reference-literal 18 features per channel and the exact float64 moments.
Run:  python tests/golden/make_aux_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import reference_ops as ro  # noqa: E402

# one intensity per type, taken from the reference's sweep (experiments/*: datasets_<type>_<I>)
NOISE_CASES = {"gaussian": 30, "salt_and_pepper": 15, "speckle": 35, "poisson": 60, "uniform": 25}


def noise():
    x = np.random.default_rng(0).integers(0, 256, (2, 32, 32, 3), dtype=np.uint8)
    for k, (t, inten) in enumerate(NOISE_CASES.items()):
        np.random.seed(100 + k)
        draws = [ro.draw(t, img, inten) for img in x]
        ref = np.stack([ro.apply(t, img, inten, d) for img, d in zip(x, draws)])
        d = dict(x=x, ref=ref, intensity=inten)
        if t == "salt_and_pepper":
            d["salt"] = np.stack([dd[0] for dd in draws])
            d["pepper"] = np.stack([dd[1] for dd in draws])
        else:
            d["draws"] = np.stack(draws)
        np.savez_compressed(os.path.join(HERE, f"noise_{t}.npz"), **d)
        print(t, ref.shape)


def advstats():
    rng = np.random.default_rng(1)
    cases = {}
    cases["rgb64_a"] = rng.integers(0, 256, (3, 64, 64), dtype=np.uint8)
    cases["rgb64_b"] = rng.integers(0, 256, (3, 64, 64), dtype=np.uint8)
    yy, xx = np.mgrid[0:64, 0:64]
    stripes = ((np.sin(xx / 3.0) + np.cos(yy / 5.0)) * 60 + 128).astype(np.uint8)
    cases["struct64"] = np.stack([stripes, (xx * 4 % 256).astype(np.uint8), np.full((64, 64), 7, np.uint8)])
    cases["odd37x53"] = rng.integers(0, 256, (3, 37, 53), dtype=np.uint8)
    cases["gray128"] = rng.integers(0, 256, (1, 128, 128), dtype=np.uint8)
    out = {}
    for name, u8 in cases.items():
        x = u8.astype(np.float32) / 255.0
        out[name + "_u8"] = u8
        out[name + "_ref"] = ro.extract_advanced_features(x)
        out[name + "_f64"] = ro.advanced_moments_f64(x)
        print(name, u8.shape)
    np.savez_compressed(os.path.join(HERE, "advstats.npz"), **out)


if __name__ == "__main__":
    noise()
    advstats()
