"""Parity metrics shared by the tests.

Two bars, both TOL = 1e-5 (BASELINE.json north_star: "coefficients within 1e-5 rel of the
reference"):

1. per coefficient index k:  err[k] = max |S_gpu - S_ref|[k] / max |S_ref[k]|, maxima over every
   plane and spatial position that carries coefficient k.  Real WST coefficients span ~3
   decades (S0 ~ 0.5, S2 ~ 5e-4), so a flat elementwise relative bound over all
   entries is ill-posed in fp32; the per-k normalisation is the main contract.
2. elementwise, on the significant entries only: |S_gpu - S_ref| / |S_ref| wherever
   |S_ref| >= 1e-3 * max |S_ref[k]| (the entries of coefficient k within three decades of its
   largest value).  This guards the small values inside each coefficient map.
"""
import numpy as np

TOL = 1e-5
SIGNIFICANT = 1e-3


def _by_coef(a, ref_shape):
    K = ref_shape[-3]
    return np.moveaxis(np.asarray(a, np.float64).reshape((-1,) + tuple(ref_shape[-3:])), 1, 0).reshape(K, -1)


def per_coef_error(got, ref, floor=0.0):
    """floor > 0: the denominator of coefficient k is at least floor x the largest |S_ref| of all
    coefficients (for inputs whose symmetry makes some coefficients exactly zero, which the float64
    oracle holds as rounding noise: those are compared at an absolute TOL * floor of the strongest
    coefficient instead of relative to their own noise)."""
    assert np.shape(got) == np.shape(ref), (np.shape(got), np.shape(ref))
    g, r = _by_coef(got, np.shape(ref)), _by_coef(ref, np.shape(ref))
    scale = np.abs(r).max(axis=1)
    scale = np.maximum(scale, floor * scale.max())
    scale = np.where(scale > 0, scale, 1.0)
    return np.abs(g - r).max(axis=1) / scale


def elementwise_error(got, ref, significant=SIGNIFICANT, floor=0.0):
    """Per coefficient k: max elementwise relative error over the entries with
    |S_ref| >= significant * max |S_ref[k]| (0 where k has no such entry); with floor > 0 only the
    coefficients whose max |S_ref[k]| reaches floor x the strongest coefficient are checked."""
    assert np.shape(got) == np.shape(ref), (np.shape(got), np.shape(ref))
    g, r = _by_coef(got, np.shape(ref)), _by_coef(ref, np.shape(ref))
    ar = np.abs(r)
    kmax = ar.max(axis=1, keepdims=True)
    lim = np.maximum(significant * kmax, np.where(kmax >= floor * kmax.max(), 0.0, np.inf))
    mask = (ar >= lim) & (ar > 0)
    rel = np.where(mask, np.abs(g - r) / np.where(mask, ar, 1.0), 0.0)
    return rel.max(axis=1)


def assert_parity(got, ref, tol=TOL, what="", elementwise=True, floor=0.0):
    err = per_coef_error(got, ref, floor)
    worst = int(np.argmax(err))
    assert err.max() <= tol, f"{what}: max per-coefficient rel err {err.max():.3e} at k={worst} (tol {tol})"
    if elementwise:
        ew = elementwise_error(got, ref, floor=floor)
        w = int(np.argmax(ew))
        assert ew.max() <= tol, (f"{what}: max elementwise rel err {ew.max():.3e} on significant entries "
                                 f"(|S_ref| >= {SIGNIFICANT:g} max|S_ref[k]|) at k={w} (tol {tol})")
    return err
