"""CPU tests of the float64 oracle (oracle/kymatio_ref.py): known answers, layout pins, and the
committed golden fixtures.  Parity with kymatio itself is unpinned."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import kymatio_ref as kr

PHI0 = np.pi / 3.1415   # kymatio normalises with the literal 3.1415


def rgb(seed, C, M, N):
    return np.random.default_rng(seed).integers(0, 256, (C, M, N)).astype(np.float32) / 255


@pytest.mark.parametrize("M,J", [(64, 2), (64, 4), (32, 3), (40, 1)])
def test_compute_padding(M, J):
    P = kr.compute_padding(M, M, J)[0]
    assert P % 2 ** J == 0 and P > M
    assert P == ((M + 2 ** J) // 2 ** J + 1) * 2 ** J


def test_padding_known_sizes():
    assert kr.compute_padding(64, 64, 2) == (72, 72)
    assert kr.compute_padding(64, 64, 4) == (96, 96)
    assert kr.compute_padding(128, 128, 2) == (136, 136)
    assert kr.compute_padding(256, 256, 6) == (384, 384)
    assert kr.compute_padding(32, 32, 3) == (48, 48)


@pytest.mark.parametrize("J,L,K", [(2, 8, 81), (4, 8, 417), (3, 6, 127), (6, 12, 2233)])
def test_num_coefficients(J, L, K):
    assert kr.num_coefficients(J, L) == K


def test_phi_dc_and_psi_zero_mean():
    for P, J in [(72, 2), (96, 4), (48, 3)]:
        fb = kr.filter_bank(P, P, J, 8)
        for lev in fb["phi"]["levels"]:
            assert abs(lev[0, 0] - PHI0) < 1e-12
        for p in fb["psi"]:
            assert abs(p["levels"][0][0, 0]) < 1e-15


def test_filter_levels_count():
    J = 4
    fb = kr.filter_bank(96, 96, J, 8)
    for p in fb["psi"]:
        assert len(p["levels"]) == min(p["j"] + 1, max(J - 1, 1))
        for r, lev in enumerate(p["levels"]):
            assert lev.shape == (96 >> r, 96 >> r)
    assert len(fb["phi"]["levels"]) == J


def test_masked_crop_matches_literal_loops():
    x = np.random.default_rng(3).standard_normal((24, 16))
    for r in range(3):
        np.testing.assert_allclose(kr.periodize_filter_fft(x, r), kr.periodize_filter_fft_loops(x, r),
                                   rtol=0, atol=1e-14)


def test_masked_crop_keeps_negative_nyquist():
    # level 1 of a length-8 spectrum keeps bins [-2, 2): index 2 of the crop is bin -2 (=6)
    x = np.zeros((8, 8))
    x[6, 0] = 1.0      # frequency -2 along rows
    x[2, 0] = 10.0     # frequency +2: zeroed by the mask
    c = kr.periodize_filter_fft(x, 1)
    assert c[2, 0] == 1.0


def test_psi_angles_match_layout_pin():
    # compare_wst_coefficients.py:55,67: angle = (int(L - L/2 - 1) - l) * pi / L
    for L in (6, 8, 12):
        for l in range(L):
            assert (int(L - L / 2 - 1) - l) * np.pi / L == pytest.approx((int(L - L / 2 - 1) - l) * np.pi / L)
    # order-1 flat index 1 + j*L + l (compare_wst_coefficients.py:63-67)
    assert kr.coefficient_index(3, 6, 2, 5) == 1 + 2 * 6 + 5
    assert kr.coefficient_index(4, 8, 0, 0, 1, 0) == 1 + 32
    assert kr.coefficient_index(4, 8, 0, 1, 1, 0) == 1 + 32 + 24


def test_constant_image_known_answer():
    S = kr.Scattering2D(J=2, shape=(64, 64), L=8)(np.full((64, 64), 0.25))
    np.testing.assert_allclose(S[0], 0.25 * PHI0, rtol=1e-12)
    assert np.abs(S[1:]).max() < 1e-14


def test_s0_affine_and_s12_shift_invariant_homogeneous():
    x = rgb(1, 1, 32, 32)[0].astype(np.float64)
    sc = kr.Scattering2D(J=2, shape=(32, 32), L=6)
    a, b = 2.5, 0.7
    S, Sab = sc(x), sc(a * x + b)
    np.testing.assert_allclose(Sab[0], a * S[0] + PHI0 * b, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Sab[1:], a * S[1:], rtol=1e-9, atol=1e-13)
    Sneg = sc(-x)
    np.testing.assert_allclose(Sneg[1:], S[1:], rtol=1e-9, atol=1e-13)


def test_batch_shape_roundtrip_and_errors():
    sc = kr.Scattering2D(J=2, shape=(32, 32), L=4)
    x = rgb(2, 6, 32, 32).reshape(2, 3, 32, 32)
    S = sc(x)
    assert S.shape == (2, 3, 1 + 8 + 16, 8, 8)
    np.testing.assert_allclose(S[1, 2], sc(x[1, 2]), rtol=1e-13)
    with pytest.raises(TypeError):
        sc([[0.0]])
    with pytest.raises(RuntimeError):
        sc(np.zeros(32))
    with pytest.raises(RuntimeError):
        sc(np.zeros((31, 32)))
    with pytest.raises(RuntimeError):
        kr.Scattering2D(J=6, shape=(32, 32))


def test_feature_layouts():
    x = rgb(4, 3, 32, 32)
    f = kr.extract_wst_features(x, J=2, L=8)
    assert f.shape == (486,)
    g = kr.extract_wst_features_interleaved(x, J=2, L=8)
    # same numbers, permuted: training [m | s] per channel vs interleaved [m0 s0 m1 s1 ...]
    ft = f.reshape(3, 2, 81)
    np.testing.assert_allclose(g.reshape(3, 81, 2), np.moveaxis(ft, 1, 2), rtol=1e-14)


def test_golden_manifest_consistent():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        man = json.load(fh)
    for name, m in man.items():
        d = load_golden(name)
        assert list(d["S"].shape) == m["out_shape"]
        assert d["S"].shape[1] == kr.num_coefficients(m["J"], m["L"], m["max_order"])


@pytest.mark.parametrize("name", ["c1_rgb64_J2_L8", "c2_rgb64_J4_L8", "cmp_gray32_J3_L6",
                                  "rect_40x56_J2_L5", "order1_rgb64_J3_L8"])
def test_oracle_reproduces_golden(name):
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        m = json.load(fh)[name]
    d = load_golden(name)
    x = d["x_u8"].astype(np.float32) / 255
    S = kr.Scattering2D(J=m["J"], shape=(m["M"], m["N"]), L=m["L"], max_order=m["max_order"])(x)
    np.testing.assert_allclose(S.astype(np.float32), d["S"], rtol=2e-6, atol=1e-9)


def test_oracle_reproduces_pattern_golden():
    """The c5-geometry structured-pattern fixture (tests/golden/make_pattern_golden.py) is the
    oracle's output: re-run one plane (the impulse, ~4 s)."""
    d = load_golden("c5_patterns_256_J6_L12")
    names = [str(n) for n in d["names"]]
    i = names.index("impulse")
    S = kr.Scattering2D(J=int(d["J"]), shape=d["x"].shape[-2:], L=int(d["L"]))(d["x"][i:i + 1])
    np.testing.assert_allclose(S[0].astype(np.float32), d["S"][i], rtol=2e-6, atol=1e-9)


def test_real_data_magnitude_sanity():
    # real 128^2 patches (J=2, L=8) have mean S0 ~ 0.5-0.63, S1 ~ 5e-3, S2 ~ 5e-4.
    # A uniform-noise 64^2 patch must land in the same decades for S0 and be non-trivial for S1/S2.
    d = load_golden("c1_rgb64_J2_L8")
    S = d["S"].astype(np.float64)
    assert 0.3 < S[:, 0].mean() < 0.7
    assert 1e-4 < S[:, 1:17].mean() < 0.2
    assert 1e-6 < S[:, 17:].mean() < S[:, 1:17].mean()


@pytest.mark.parametrize("M,J,L", [(64, 4, 8), (128, 2, 8), (32, 3, 6)])
def test_grid_symmetries_permute_orientations(M, J, L):
    """SURVEY §4.4 rotation pin: rot90 permutes the orientation indices by L/2 (mod L), a row flip
    by l -> L-2-l, a transpose by l -> L/2-2-l; S2 permutes in theta1 and theta2 (tests/symmetry.py)."""
    from symmetry import exact_mask, grid_ops, symmetry_errors
    s = kr.Scattering2D(J=J, shape=(M, M), L=L, pre_pad=True)
    P = s.M_padded
    x = np.random.default_rng(7).random((2, P, P))
    Sx = s(x)
    exact = exact_mask(J, L)
    for name, (op, f, mapop) in grid_ops(P, J, L).items():
        err = symmetry_errors(Sx, s(op(x)), J, L, f, mapop)
        assert err[exact].max() < 1e-12, (name, err[exact].max())
        if (~exact).any():
            # level-j1 >= 1 crops of the masked periodisation keep only the negative Nyquist bin
            assert 1e-6 < err[~exact].max() < 3e-3, (name, err[~exact].max())
