"""CPU tests of rows F2 / F4 (no GPU): the oracle restatements against the committed fixtures
and the reference's conventions, feature-name layouts, and the C ABI's host-side helpers."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import reference_ops as ro

import wst_amd  # noqa: F401
from wst_amd import _lib, features


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("t", ro.NOISE_TYPES)
def test_noise_oracle_reproduces_fixture(t):
    d = load(f"noise_{t}.npz")
    x, ref, inten = d["x"], d["ref"], float(d["intensity"])
    for i in range(x.shape[0]):
        dr = (d["salt"][i], d["pepper"][i]) if t == "salt_and_pepper" else d["draws"][i]
        np.testing.assert_array_equal(ro.apply(t, x[i], inten, dr), ref[i])


def test_salt_pepper_conventions():
    d = load("noise_salt_and_pepper.npz")
    ns, npp = ro.salt_and_pepper_counts((32, 32, 3), 15)
    assert d["salt"].shape == (2, 2, ns) and d["pepper"].shape == (2, 2, npp)
    # randint(0, dim - 1): the last row / column is never hit (add_noise.py:31,37)
    assert d["salt"].max() <= 30 and d["pepper"].max() <= 30
    x, ref = d["x"], d["ref"]
    changed = np.any(ref != x, axis=-1)
    assert not changed[:, -1, :].any() and not changed[:, :, -1].any()
    # every channel of a hit pixel is set (salt 255 / pepper 0)
    hit = ref[changed]
    assert np.all((hit == 255).all(-1) | (hit == 0).all(-1))


def test_salt_pepper_counts_abi_matches_reference():
    lib = _lib.load()
    import ctypes
    for (H, W, C, I) in [(32, 32, 3, 15), (64, 64, 3, 5), (128, 128, 3, 25), (7, 9, 1, 33.3)]:
        a, b = ctypes.c_int64(), ctypes.c_int64()
        assert lib.wst_salt_pepper_counts(H, W, C, I, ctypes.byref(a), ctypes.byref(b)) == 0
        assert (a.value, b.value) == ro.salt_and_pepper_counts((H, W, C), I)


def test_advanced_oracle_against_fixture_and_f64():
    d = load("advstats.npz")
    for name in ("rgb64_a", "struct64", "odd37x53", "gray128"):
        x = d[name + "_u8"].astype(np.float32) / 255.0
        np.testing.assert_array_equal(ro.extract_advanced_features(x), d[name + "_ref"])
        f = d[name + "_ref"].reshape(-1, 18)
        f64 = d[name + "_f64"]
        # the reference's float32 moments agree with exact ones to float32 cancellation level
        ok = np.isfinite(f64[:, 3])
        np.testing.assert_allclose(f[ok][:, [0, 1, 2, 8, 15]], f64[ok][:, [0, 1, 2, 5, 6]], rtol=2e-6)
        np.testing.assert_allclose(f[ok][:, 6], f64[ok][:, 3], rtol=1e-3, atol=1e-4)


def test_feature_names_match_reference_layouts():
    ref = json.load(open(os.path.join(GOLDEN, "ref_feature_names.json")))
    assert features.get_feature_names("hybrid") == ref["hybrid"]
    assert features.get_feature_names("wst") == ref["wst"]
    adv = features.get_feature_names("advanced_stats")
    assert len(adv) == 54 and adv[:2] == ["R_mean", "R_std"] and adv[-1] == "B_edge_density"
    with pytest.raises(ValueError):
        features.get_feature_names("pixels")
