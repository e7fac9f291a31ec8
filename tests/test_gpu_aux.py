"""GPU parity of rows F2 (noise injection, add_noise.py:14-72) and F4 (advanced_stats,
train_and_save_model.py:58-112) through the C ABI (csrc/wst_aux.hip).

Bars (written here):
* noise formulas on the reference's own draws: bit-exact uint8 (and float32 CHW == uint8 / 255);
* Philox production draws: distribution checks (moments within 5 standard errors), clipping,
  salt & pepper counts / last row-column convention, determinism per seed;
* advanced_stats: min/max/range/percentiles/iqr/edge_density bit-exact with numpy / scipy's
  float32 arithmetic; the moment features within 1e-9 relative of their exact (float64) values
  and within the reference's own float32 error of the reference-literal values (2e-6 relative;
  skew / kurtosis 1e-3 relative + 1e-4 absolute); grad_mean within 1e-6 relative (the
  reference sums float32 magnitudes pairwise).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import reference_ops as ro

import wst_amd  # noqa: F401
from wst_amd import features, noise

pytestmark = pytest.mark.gpu
EXACT = [3, 4, 5, 9, 10, 11, 12, 13, 14, 17]
MOM = list(ro.MOMENT_IDX)


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("t", ro.NOISE_TYPES)
def test_noise_formulas_bit_exact_on_reference_draws(t):
    d = load(f"noise_{t}.npz")
    x, ref, inten = d["x"], d["ref"], float(d["intensity"])
    draws = (d["salt"], d["pepper"]) if t == "salt_and_pepper" else d["draws"]
    got = noise.apply_noise_draws(x, t, inten, draws).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    chw = noise.apply_noise_draws(x, t, inten, draws, out="float_chw").cpu().numpy()
    np.testing.assert_array_equal(chw, np.transpose(ref, (0, 3, 1, 2)).astype(np.float32) / 255.0)


def test_philox_noise_distributions():
    B, H, W, C = 64, 64, 64, 3
    x = np.full((B, H, W, C), 128, np.uint8)
    # gaussian I=30 -> sigma = 76.5; far from the clip bounds only at small sigma: use I=5
    g = noise.add_noise_batch(x, "gaussian", 5, seed=1).double() - 128
    sig = 5 * 255 / 100
    n = g.numel()
    # truncation to uint8 biases the mean by ~ -0.5
    assert abs(g.mean().item() + 0.5) < 5 * sig / n ** 0.5 + 0.01
    assert abs(g.std().item() - (sig ** 2 + 1 / 12) ** 0.5) < 0.02 * sig
    u = noise.add_noise_batch(x, "uniform", 40, seed=2).double() - 128
    r = 40 * 255 / 100
    assert u.min().item() >= -r / 2 - 1 and u.max().item() <= r / 2
    assert abs(u.std().item() - (r * r / 12 + 1 / 12) ** 0.5) < 0.02 * r
    # poisson: lambda = 128 * sf / 255; output = k * 255 / sf truncated
    p = noise.add_noise_batch(x, "poisson", 60, seed=3).double()
    sf = ro.poisson_scale(60)
    lam = 128 * sf / 255
    k_est = p.mean().item() * sf / 255
    assert abs(k_est - lam) < 0.05 * lam
    # determinism and seed dependence
    a = noise.add_noise_batch(x, "speckle", 35, seed=4)
    b = noise.add_noise_batch(x, "speckle", 35, seed=4)
    c = noise.add_noise_batch(x, "speckle", 35, seed=5)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert not torch.equal(a[0], a[1]), "images of a batch must get independent draws"


def test_philox_salt_and_pepper_conventions():
    B, H, W, C = 8, 32, 32, 3
    x = np.full((B, H, W, C), 100, np.uint8)
    y = noise.add_noise_batch(x, "salt_and_pepper", 25, seed=7).cpu().numpy()
    ns, npp = noise.salt_pepper_counts(H, W, C, 25)
    changed = np.any(y != 100, axis=-1)
    assert not changed[:, -1, :].any() and not changed[:, :, -1].any()
    hit = y[changed]
    assert np.all((hit == 255).all(-1) | (hit == 0).all(-1))
    # distinct coordinates hit <= draws; with 1/961 collision odds most land distinct
    per = changed.reshape(B, -1).sum(1)
    assert np.all(per <= ns + npp) and np.all(per > 0.6 * (ns + npp))


def test_advanced_stats_parity():
    d = load("advstats.npz")
    for name in ("rgb64_a", "rgb64_b", "struct64", "odd37x53", "gray128"):
        u8 = d[name + "_u8"]
        x = u8.astype(np.float32) / 255.0
        got = features.extract_advanced_features_batch(x[None])[0].reshape(-1, 18)
        ref = d[name + "_ref"].reshape(-1, 18)
        f64 = d[name + "_f64"]
        np.testing.assert_array_equal(got[:, EXACT], ref[:, EXACT], err_msg=name)
        ok = np.isfinite(f64[:, 3])
        np.testing.assert_allclose(got[:, MOM][ok], f64[ok], rtol=1e-9, atol=1e-12, err_msg=name)
        assert np.all(np.isnan(got[~ok][:, [6, 7]])), "constant channel: skew/kurt NaN (scipy rule)"
        np.testing.assert_allclose(got[ok][:, [0, 1, 2, 8, 15]], ref[ok][:, [0, 1, 2, 8, 15]],
                                   rtol=2e-6, err_msg=name)
        np.testing.assert_allclose(got[ok][:, [6, 7]], ref[ok][:, [6, 7]], rtol=1e-3, atol=1e-4,
                                   err_msg=name)
        np.testing.assert_allclose(got[:, 16], ref[:, 16], rtol=1e-6, err_msg=name)


def test_advanced_stats_batch_and_hybrid_layout():
    d = load("advstats.npz")
    a = d["rgb64_a_u8"].astype(np.float32) / 255.0
    b = d["rgb64_b_u8"].astype(np.float32) / 255.0
    got = features.extract_advanced_features_batch(np.stack([a, b, a]))
    np.testing.assert_array_equal(got[0], got[2])
    np.testing.assert_array_equal(got[1], features.extract_advanced_features(b))
    h = features.extract_hybrid_features(a)
    assert h.shape == (54 + 486,)
    np.testing.assert_array_equal(h[:54], got[0])
    np.testing.assert_array_equal(h[54:], features.extract_wst_features(a))
    assert features.extract_features(a, "hybrid").shape == (540,)


def test_noise_to_wst_pipeline_matches_host_composition():
    """c4 data path: noisy uint8 -> float32 CHW / 255 on the device -> pooled WST features, equal
    to running the same noisy uint8 images through the host-side conversion + features."""
    x = np.random.default_rng(9).integers(0, 256, (4, 64, 64, 3), dtype=np.uint8)
    chw = noise.add_noise_batch(x, "gaussian", 30, seed=11, out="float_chw")
    u8 = noise.add_noise_batch(x, "gaussian", 30, seed=11).cpu().numpy()
    host = np.transpose(u8, (0, 3, 1, 2)).astype(np.float32) / 255.0
    np.testing.assert_array_equal(chw.cpu().numpy(), host)
    f_dev = features.extract_wst_features_batch(chw, J=4, L=8)
    f_host = features.extract_wst_features_batch(host, J=4, L=8)
    np.testing.assert_array_equal(f_dev, f_host)
