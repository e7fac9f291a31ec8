"""Generate the golden fixtures under tests/golden/ from the float64 oracle.

Parity with kymatio itself is unpinned (kymatio is absent and the reference cannot be executed,
SURVEY.md §8(c)); these vectors freeze the oracle's output on fixed seeded inputs so that the GPU
tests do not need /root/reference or the oracle's run time at test time, and so that any future
change to the oracle shows up as a fixture diff.

Inputs mimic load_rgb_image (train_and_save_model.py:51-56): uint8 k/255, seed 0.
Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import kymatio_ref as kr  # noqa: E402

# name: (C, M, N, J, L, max_order, note)
CASES = {
    "c1_rgb64_J2_L8": (3, 64, 64, 2, 8, 2, "BASELINE config 1: one 64x64 RGB patch, J=2 L=8"),
    "c2_rgb64_J4_L8": (3, 64, 64, 4, 8, 2, "BASELINE config 2 geometry: 64x64 RGB, J=4 L=8"),
    "cmp_gray32_J3_L6": (1, 32, 32, 3, 6, 2, "compare_wst_coefficients.py:35-39 (32x32, J=3, L=6)"),
    "rect_40x56_J2_L5": (2, 40, 56, 2, 5, 2, "non-square, odd L"),
    "order1_rgb64_J3_L8": (3, 64, 64, 3, 8, 1, "max_order=1"),
    "f3_rgb128_J2_L8": (1, 128, 128, 2, 8, 2, "reference real geometry 128x128 J=2 (P=136), 1 channel"),
    "c5_ms256_J6_L12": (1, 256, 256, 6, 12, 2, "BASELINE config 5 geometry, 1 band"),
    "staged192_gray128_J5_L8": (1, 128, 128, 5, 8, 2, "P=192: one HBM-staged level (192^2) then LDS levels"),
    "staged384_gray256_J6_L7": (1, 256, 256, 6, 7, 2, "two HBM-staged levels (384^2, 192^2), odd L: the "
                                "all-paths s = 2 row pass with an unpaired last path"),
    "rectstaged_256x128_J4_L8": (1, 256, 128, 4, 8, 2, "rectangular plane needing a staged level (288 x 160)"),
    "staged224_gray192_J4_L8": (1, 192, 192, 4, 8, 2, "P=224 (family 7): staged level size 224"),
}


def make(name, C, M, N, J, L, max_order):
    rng = np.random.default_rng(0)
    x8 = rng.integers(0, 256, (C, M, N), dtype=np.uint8)
    x = x8.astype(np.float32) / 255.0
    S = kr.Scattering2D(J=J, shape=(M, N), L=L, max_order=max_order)(x)
    feats = kr.extract_wst_features(x, J=J, L=L) if (C == 3 and max_order == 2) else None
    d = dict(x_u8=x8, S=S.astype(np.float32), S_absmax=np.abs(S).reshape(C, S.shape[1], -1).max(-1),
             J=J, L=L, max_order=max_order)
    if feats is not None:
        d["features_train"] = feats
        d["features_interleaved"] = kr.extract_wst_features_interleaved(x, J=J, L=L)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    return S.shape


def main(names=None):
    manifest = {}
    if names and os.path.exists(os.path.join(HERE, "manifest.json")):
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
    for name, (C, M, N, J, L, mo, note) in CASES.items():
        if names and name not in names:
            continue
        shape = make(name, C, M, N, J, L, mo)
        manifest[name] = dict(C=C, M=M, N=N, J=J, L=L, max_order=mo, out_shape=list(shape),
                              note=note, seed=0, generator="oracle/kymatio_ref.py (float64)")
        print(name, shape, flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
