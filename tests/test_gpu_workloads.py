"""GPU tests of the c3 and c4 workloads of BASELINE.json against the kymatio oracle.

* c3 (1M synthetic 64x64 RGB patches sharded over GPUs): patches are generated on the device by
  (seed, global patch index) -- ``wst_patch_generate``, pinned bit-exactly to its host
  restatement ``oracle/patchgen.py`` (Philox4x32-10, Random123 known answers in
  tests/test_bench_cpu.py) -- and transformed by ``distributed.extract_sharded`` with its
  default HIP compute.  64 sampled global indices are recreated on the host and checked against
  ``kymatio_ref.extract_wst_features`` (train_and_save_model.py:346-378).
* c4 (noise-robustness sweep at J=4, L=8): each of the 13 (type, intensity) cases of
  bench.py NOISE_SWEEP gets the reference's own numpy draws (add_noise.py:14-72 via
  oracle/reference_ops.py), goes through ``wst_noise_apply`` -> float32 CHW / 255 on the device
  -> pooled WST features, and is compared with the oracle run on the reference's noisy uint8.

Tolerance (pooled features; tests/parity.py): per feature index f, max over the images of
|F_gpu - F_ref| / max |F_ref| <= 1e-5.
"""
import numpy as np
import pytest
import torch

from oracle import kymatio_ref as kr
from oracle import patchgen
from oracle import reference_ops as ro
from parity import TOL

import wst_amd  # noqa: F401
from wst_amd import data, distributed, features, noise

pytestmark = pytest.mark.gpu

NOISE_SWEEP = [("gaussian", 30), ("gaussian", 50), ("poisson", 40), ("poisson", 60),
               ("salt_and_pepper", 5), ("salt_and_pepper", 15), ("salt_and_pepper", 25),
               ("speckle", 15), ("speckle", 35), ("speckle", 55),
               ("uniform", 10), ("uniform", 25), ("uniform", 40)]


def feature_error(got, ref):
    got = np.asarray(got, np.float64).reshape(-1, np.shape(ref)[-1])
    ref = np.asarray(ref, np.float64).reshape(got.shape)
    scale = np.abs(ref).max(axis=0)
    scale = np.where(scale > 0, scale, 1.0)
    return (np.abs(got - ref).max(axis=0) / scale).max()


def test_patch_generator_matches_host_restatement():
    first, n = 999_000, 7           # indices near the end of c3's 1M range, odd count
    got = data.generate_patches(1, first, n, 3, 64, 64, out="uint8").cpu().numpy()
    ref = patchgen.generate_patches_u8(1, first, n, 3, 64, 64)
    np.testing.assert_array_equal(got, ref)
    f = data.generate_patches(1, first, n, 3, 64, 64).cpu().numpy()
    np.testing.assert_array_equal(f, ref.astype(np.float32) / 255.0)
    # a patch's bytes do not depend on how the range is split (world size / chunking)
    a = data.generate_patches(1, first, 3, 3, 64, 64, out="uint8")
    b = data.generate_patches(1, first + 3, n - 3, 3, 64, 64, out="uint8")
    np.testing.assert_array_equal(torch.cat([a, b]).cpu().numpy(), ref)
    # odd element counts (per-patch tail shorter than one 16-byte Philox block)
    odd = data.generate_patches(5, 12345, 3, 1, 5, 7, out="uint8").cpu().numpy()
    np.testing.assert_array_equal(odd, patchgen.generate_patches_u8(5, 12345, 3, 1, 5, 7))


def test_c3_sharded_hip_compute_64_sampled_patches_vs_oracle():
    total, first, n = 1_000_000, 1_000_000 - 512, 512   # the last 512 patches of c3's range
    x = data.generate_patches(1, first, n, 3, 64, 64)
    F = distributed.extract_sharded(x, J=4, L=8)                     # default HIP compute
    F = F.cpu().numpy() if torch.is_tensor(F) else np.asarray(F)
    K = kr.num_coefficients(4, 8)
    assert F.shape == (n, 3, 2 * K)
    idx = np.sort(np.random.default_rng(2024).choice(n, 64, replace=False))
    sc = kr.Scattering2D(J=4, shape=(64, 64), L=8)
    ref = []
    for i in idx:
        u8 = patchgen.generate_patches_u8(1, first + int(i), 1, 3, 64, 64)[0]
        ref.append(kr.extract_wst_features(u8.astype(np.float32) / 255, J=4, L=8, scattering=sc))
    ref = np.stack(ref)
    err = feature_error(F[idx].reshape(64, -1), ref)
    assert err <= TOL, f"c3 sampled patches: max per-feature rel err {err:.3e}"
    assert first + n == total


@pytest.mark.parametrize("ntype,intensity", NOISE_SWEEP)
def test_c4_noise_case_vs_oracle(ntype, intensity):
    rng = np.random.default_rng(100 + intensity)
    imgs = rng.integers(0, 256, (2, 64, 64, 3), dtype=np.uint8)
    np.random.seed(7 * intensity + len(ntype))          # the reference draws from numpy's global RNG
    draws = [ro.draw(ntype, im, intensity) for im in imgs]
    noisy_ref = np.stack([ro.apply(ntype, im, intensity, d) for im, d in zip(imgs, draws)])
    if ntype == "salt_and_pepper":
        dd = (np.stack([d[0] for d in draws]), np.stack([d[1] for d in draws]))
    else:
        dd = np.stack(draws)
    u8 = noise.apply_noise_draws(imgs, ntype, intensity, dd).cpu().numpy()
    np.testing.assert_array_equal(u8, noisy_ref)                      # formulas bit-exact
    chw = noise.apply_noise_draws(imgs, ntype, intensity, dd, out="float_chw")
    got = features.extract_wst_features_batch(chw, J=4, L=8)
    sc = kr.Scattering2D(J=4, shape=(64, 64), L=8)
    ref = np.stack([kr.extract_wst_features(np.transpose(im, (2, 0, 1)).astype(np.float32) / 255,
                                            J=4, L=8, scattering=sc) for im in noisy_ref])
    err = feature_error(got, ref)
    assert err <= TOL, f"{ntype} {intensity}: max per-feature rel err {err:.3e}"


def test_u8_hwc_to_chw_ingest():
    rng = np.random.default_rng(3)
    for shape in [(4, 128, 128, 3), (3, 37, 53, 3), (2, 64, 64, 4), (1, 5, 3, 1)]:
        x = rng.integers(0, 256, shape, dtype=np.uint8)
        got = data.u8_hwc_to_chw(x).cpu().numpy()
        ref = np.transpose(x, (0, 3, 1, 2)).astype(np.float32) / 255.0   # load_rgb_image
        np.testing.assert_array_equal(got, ref)
