"""GPU parity on structured inputs (the synthetic patterns the reference's
visualisation uses, src/visualization/visualize_features.py:50-120 -- gradients, checkerboard,
concentric circles, random and striped textures, a sharp-edged square -- plus an impulse), at the
reference's experiment geometry (128^2, J=2, L=8) and the headline's (64^2, J=4, L=8), against the
float64 oracle.

Bars (tests/parity.py):
* per coefficient k, max|S_gpu - S_ref|[k] / max|S_ref[k]| <= 1e-5 -- strict, for every pattern
  (gradients: the denominator floored at 1e-3 of the strongest coefficient, see below);
* elementwise on the significant entries (|S_ref| >= 1e-3 max|S_ref[k]|): <= 1e-5, or, where the
  same cascade computed in fp32 by scipy's pocketfft (the reference's own algorithm, only the dtype
  changed: ``fp32_cascade``) cannot meet 1e-5 itself, <= 2x that fp32 pipeline's error on the same
  plane.  An fp32 FFT's error is absolute (~1e-7 of the map's largest value), so on flat/edged
  inputs an entry three decades below its map's peak carries ~1e-4 relative error in ANY fp32
  implementation: measured the fp32 pocketfft pipeline reaches 5.5e-4 on the
  gradients and 2-4e-4 on the edge, and even exceeds the per-coefficient 1e-5 bar on the gradients
  (1.7e-5), which the HIP path holds.

The generators below are this repository's own restatement of those pattern definitions (input
data only).  They exercise what random uint8 noise does not: constant rows / columns meeting the
reflect padding (gradients), energy concentrated at the highest frequencies (checkerboard), a
single bin (impulse) and large flat regions with sharp edges.
"""
import numpy as np
import pytest

from oracle import kymatio_ref as kr
from parity import TOL, assert_parity, elementwise_error

from wst_amd.numpy import Scattering2D as NpS

pytestmark = pytest.mark.gpu


def patterns(n):
    t = np.linspace(0.0, 1.0, n)
    out = {
        "gradient_h": np.tile(t, (n, 1)),
        "gradient_v": np.tile(t[:, None], (1, n)),
    }
    sq = n // 8
    ij = np.add.outer(np.arange(n) // sq, np.arange(n) // sq)
    out["checkerboard"] = (ij % 2 == 0).astype(np.float64)
    yy, xx = np.mgrid[0:n, 0:n]
    r = np.hypot(yy - n / 2, xx - n / 2) / (n / 2)
    out["circles"] = np.sin(r * 5 * np.pi) * 0.5 + 0.5
    rng = np.random.RandomState(42)
    out["texture"] = rng.rand(n, n)
    stripes = (np.sin(np.linspace(0, 8 * 2 * np.pi, n))[None, :].repeat(n, 0) + 1) / 2
    out["vertical_texture"] = np.clip(stripes * 0.7 + rng.rand(n, n) * 0.3, 0, 1)
    edge = np.zeros((n, n))
    b = n * 20 // 128
    edge[b:n - b, b:n - b] = 1.0
    out["edge"] = edge
    imp = np.zeros((n, n))
    imp[n // 3, n // 2] = 1.0
    out["impulse"] = imp
    return {k: v.astype(np.float32) for k, v in out.items()}


def fp32_cascade(sc, x):
    """The oracle's cascade (kymatio_ref.scattering2d) run with float32 input and filters, so every
    FFT is scipy's single-precision pocketfft: the fp32 noise floor of the reference algorithm."""
    def f32(d):
        return {**d, "levels": [np.asarray(v, np.float32) for v in d["levels"]]}
    out = kr.scattering2d(np.asarray(x, np.float32), lambda v: kr.reflect_pad(v, sc.pad_size),
                          sc.J, sc.L, f32(sc.phi), [f32(p) for p in sc.psi], sc.max_order)
    assert out.dtype == np.float32
    return out


@pytest.mark.parametrize("n,J", [(128, 2), (64, 4)])
def test_structured_patterns_against_oracle(n, J):
    pats = patterns(n)
    x = np.stack(list(pats.values()))                 # (8, n, n): one plane per pattern
    got = NpS(J=J, shape=(n, n), L=8)(x)
    sc = kr.Scattering2D(J=J, shape=(n, n), L=8)
    ref = sc(x)
    f32 = fp32_cascade(sc, x)
    for i, name in enumerate(pats):
        what = f"{name} {n}x{n} J={J}"
        # a gradient is constant along one axis: the wavelets that see no variation give
        # coefficients that are exactly zero (the oracle holds 1e-17 noise, fp32 ~1e-8 of the
        # strongest coefficient), compared at an absolute 1e-8 of the strongest (floor 1e-3)
        floor = 1e-3 if name.startswith("gradient") else 0.0
        g, r = got[i:i + 1], ref[i:i + 1]
        assert_parity(g, r, what=what, floor=floor, elementwise=False)
        ew = elementwise_error(g, r, floor=floor).max()
        bar = max(TOL, 2.0 * elementwise_error(f32[i:i + 1], r, floor=floor).max())
        assert ew <= bar, f"{what}: elementwise {ew:.3e} > bar {bar:.3e} (fp32 pocketfft x2 or 1e-5)"
