"""Parity metric shared by the tests.

Per coefficient index k:  err[k] = max |S_gpu - S_ref|[k] / max |S_ref[k]|, maxima over every
plane and spatial position that carries coefficient k.  Real WST coefficients span ~3 decades
(S0 ~ 0.5, S2 ~ 5e-4), so a flat elementwise relative bound is ill-posed in fp32;
the per-k normalisation is the stated contract.  The bar is TOL = 1e-5 (BASELINE.json
north_star: "coefficients within 1e-5 rel of the reference").
"""
import numpy as np

TOL = 1e-5


def per_coef_error(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    K = ref.shape[-3]
    g = np.moveaxis(got.reshape((-1,) + ref.shape[-3:]), 1, 0).reshape(K, -1)
    r = np.moveaxis(ref.reshape((-1,) + ref.shape[-3:]), 1, 0).reshape(K, -1)
    scale = np.abs(r).max(axis=1)
    scale = np.where(scale > 0, scale, 1.0)
    return np.abs(g - r).max(axis=1) / scale


def assert_parity(got, ref, tol=TOL, what=""):
    err = per_coef_error(got, ref)
    worst = int(np.argmax(err))
    assert err.max() <= tol, f"{what}: max per-coefficient rel err {err.max():.3e} at k={worst} (tol {tol})"
    return err
