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

The generators (tests/patterns.py) are this repository's own restatement of those pattern
definitions (input data only).

At BASELINE config 5's geometry (256^2, J=6, L=12) the box-sparse folds keep only 1-2 % of the alias
taps (bins below kBoxThreshold = 1e-8 of a filter's maximum are skipped): the structured planes there
come from a committed golden (tests/golden/make_pattern_golden.py) that
also holds the fp32 pocketfft cascade's error on each plane, and run with the same bars.
"""
import os

import numpy as np
import pytest

from oracle import kymatio_ref as kr
from parity import TOL, assert_parity, elementwise_error, per_coef_error
from patterns import fp32_cascade, patterns

from wst_amd.numpy import Scattering2D as NpS

pytestmark = pytest.mark.gpu


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


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_structured_patterns_c5_geometry():
    """BASELINE config 5 geometry (one band of 256^2, J=6, L=12: levels 384^2 / 192^2 HBM-staged,
    folds at s = 16 / 32 keeping 1-2 % of the alias taps) on the gradients, checkerboard, edge and
    impulse, with the bars of test_structured_patterns_against_oracle -- except that on the edge
    the reference algorithm computed in fp32 (scipy pocketfft) itself misses the per-coefficient
    1e-5 (1.7e-5, a coefficient whose map is mostly flat): there the bar is that fp32 error."""
    d = np.load(os.path.join(GOLDEN, "c5_patterns_256_J6_L12.npz"))
    x, ref = d["x"], d["S"].astype(np.float64)
    got = NpS(J=int(d["J"]), shape=x.shape[-2:], L=int(d["L"]))(x)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    for i, name in enumerate(str(n) for n in d["names"]):
        what = f"{name} 256x256 J=6 L=12"
        floor = 1e-3 if name.startswith("gradient") else 0.0
        g, r = got[i:i + 1], ref[i:i + 1]
        # per coefficient: 1e-5, or where the reference algorithm in fp32 (pocketfft) misses 1e-5
        # itself on this plane (the edge: 1.7e-5), no worse than it
        pbar = max(TOL, float(d["f32_per_coef"][i].max()))
        pc = per_coef_error(g, r, floor).max()
        assert pc <= pbar, f"{what}: per-coefficient {pc:.3e} > bar {pbar:.3e} (1e-5 or fp32 pocketfft)"
        ew = elementwise_error(g, r, floor=floor).max()
        bar = max(TOL, 2.0 * float(d["f32_elementwise"][i].max()))
        print(f"{what}: per-coefficient {pc:.2e} (bar {pbar:.2e}), elementwise {ew:.2e} (bar {bar:.2e})")
        assert ew <= bar, f"{what}: elementwise {ew:.3e} > bar {bar:.3e} (fp32 pocketfft x2 or 1e-5)"
