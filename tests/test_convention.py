"""The recalled kymatio constants (FilterConvention / wst_filter_convention) -- CPU tests.

kymatio 0.3.0 is not in the container, so four constants of its filter construction are
recalled from upstream rather than read (VERDICT r1 "weak" #1, r2 "next" #7): the literal 3.1415
of gabor_2d's normaliser, the 5x5 periodisation grid, the gabor accumulator dtype and the dtype
of its rotation matrices R / R_inv.  They live in one
struct shared by the oracle (oracle/kymatio_ref.py FilterConvention) and the library
(wst_filter_convention, a plan parameter).  These tests

1. pin that the switch is really shared: the library's host filter bank built under each
   alternative equals the oracle's under the same alternative;
2. measure how far each alternative moves the coefficients relative to the 1e-5 parity bar
   (per-coefficient max-normalised error, tests/parity.py).  Measured (64x64, J=2/4, L=8):
   norm_pi = pi moves S0 / S1 / S2 by 2.95e-5 / 5.90e-5 / 8.85e-5 (an exact rescale by
   (3.1415/pi)^order: 3x / 6x / 9x the bar); the periodisation half-width 1 / 3 instead of 2 by
   < 1e-13; a complex64 gabor accumulator by < 1e-6; float32 rotation matrices by 1.2e-7 (S2).  So parity hinges on one constant, and a
   wrong guess for it would show as a uniform per-order scale, not as a shape error.
"""
from dataclasses import replace

import numpy as np
import pytest

from oracle import kymatio_ref as kr
from parity import TOL, per_coef_error

from wst_amd import _lib

ALTS = {
    "np.pi": replace(kr.KYMATIO_0_3_0, norm_pi=np.pi),
    "grid 3x3": replace(kr.KYMATIO_0_3_0, periodize_half=1),
    "grid 7x7": replace(kr.KYMATIO_0_3_0, periodize_half=3),
    "float32 R": replace(kr.KYMATIO_0_3_0, rot_dtype=np.float32),
}


def test_default_convention_is_the_recalled_one():
    c = _lib.default_convention()
    assert c.norm_pi == kr.KYMATIO_0_3_0.norm_pi == 3.1415
    assert c.periodize_half == kr.KYMATIO_0_3_0.periodize_half == 2
    assert kr.KYMATIO_0_3_0.gabor_dtype is np.complex128
    assert kr.KYMATIO_0_3_0.rot_dtype is np.float64 and c.flags == 0


@pytest.mark.parametrize("alt", sorted(ALTS) + ["default"])
def test_library_filters_follow_the_shared_convention(alt):
    conv = ALTS.get(alt, kr.KYMATIO_0_3_0)
    M, N, J, L = 24, 40, 3, 4
    PM, PN = kr.compute_padding(M, N, J)
    fb = kr.filter_bank(PM, PN, J, L, conv)
    for j in range(J):
        for l in range(L):
            for r, ref in enumerate(fb["psi"][j * L + l]["levels"]):
                got = _lib.host_filter(M, N, J, L, 0, j, l, r, ref.size, conv).reshape(ref.shape)
                np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    for r, ref in enumerate(fb["phi"]["levels"]):
        got = _lib.host_filter(M, N, J, L, 1, 0, 0, r, ref.size, conv).reshape(ref.shape)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


def test_bad_convention_rejected():
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(32, 32, 2, 8, 0, 0, 0, 0, 40 * 40, _lib.Convention(norm_pi=-1.0))
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(32, 32, 2, 8, 0, 0, 0, 0, 40 * 40, _lib.Convention(periodize_half=9))
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(32, 32, 2, 8, 0, 0, 0, 0, 40 * 40, _lib.Convention(flags=2))


def _orders(err, J, L):
    return err[0], err[1:1 + J * L].max(), err[1 + J * L:].max()


@pytest.mark.parametrize("J", [2, 4])
def test_output_sensitivity_to_each_constant(J):
    L = 8
    x = np.random.default_rng(0).integers(0, 256, (64, 64), dtype=np.uint8).astype(np.float32) / 255
    ref = kr.Scattering2D(J, (64, 64), L)(x)
    sens = {}
    for name, conv in list(ALTS.items()) + [
            ("complex64 gabor", replace(kr.KYMATIO_0_3_0, gabor_dtype=np.complex64))]:
        S = kr.Scattering2D(J, (64, 64), L, convention=conv)(x)
        sens[name] = _orders(per_coef_error(S[None], ref[None]), J, L)
        print(f"J={J} {name:16s} S0 {sens[name][0]:.2e}  S1 {sens[name][1]:.2e}  "
              f"S2 {sens[name][2]:.2e}  (bar {TOL:.0e})")
    # the normaliser: an exact rescale by (3.1415 / pi)^order, above the bar at every order
    q = 1.0 - 3.1415 / np.pi
    for order, e in enumerate(sens["np.pi"]):
        assert abs(e - (1 - (1 - q) ** (order + 1))) < 1e-9, (order, e)
        assert e > TOL
    # the periodisation window and the accumulator dtype stay far below the bar
    for name in ("grid 3x3", "grid 7x7"):
        assert max(sens[name]) < 1e-12, (name, sens[name])
    assert max(sens["complex64 gabor"]) < 0.1 * TOL, sens["complex64 gabor"]
    # float32 rotation matrices: cos / sin of theta rounded in the envelope's curvature only
    # (measured: S1 / S2 move by ~1e-7 relative, two decades under the bar; S0 not at all)
    assert sens["float32 R"][0] < 1e-12, sens["float32 R"]
    assert 0 < max(sens["float32 R"]) < 0.1 * TOL, sens["float32 R"]
