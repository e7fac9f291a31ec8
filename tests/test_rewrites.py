"""CPU check of the exact algebraic rewrites the HIP kernels rely on, via a float64 numpy model
of the kernels' dataflow (tests/kernel_model.py) compared with the oracle's literal cascade."""
import numpy as np
import pytest

import kernel_model as km
from oracle import kymatio_ref as kr
from parity import per_coef_error
from wst_amd import _lib


def test_reflect_index_matches_numpy_reflect_any_width():
    for n in (1, 2, 3, 5, 8):
        a = np.arange(n)
        for p in (0, 1, 3, 7, 12):
            ref = np.pad(a, (p, p), mode="reflect")
            got = np.array([a[km.reflect_index(i - p, n)] for i in range(n + 2 * p)])
            np.testing.assert_array_equal(ref, got)


@pytest.mark.parametrize("M,N,J,L", [(64, 64, 2, 8), (64, 64, 4, 8), (32, 32, 3, 6),
                                     (40, 56, 2, 5), (16, 16, 4, 4)])
def test_kernel_dataflow_equals_kymatio_cascade(M, N, J, L):
    PM, PN = kr.compute_padding(M, N, J)
    fb = kr.filter_bank(PM, PN, J, L)
    psi = {(p["j"], p["theta"]): p["levels"] for p in fb["psi"]}
    hM = [_lib.host_filter(M, N, J, L, 2, 0, 0, r, PM >> r) for r in range(J)]
    hN = [_lib.host_filter(M, N, J, L, 3, 0, 0, r, PN >> r) for r in range(J)]
    x = np.random.default_rng(0).integers(0, 256, (M, N)).astype(np.float64) / 255
    ref = kr.Scattering2D(J=J, shape=(M, N), L=L)(x)
    got = km.scatter_model(x, J, L, hM, hN, psi)
    assert per_coef_error(got, ref).max() < 1e-12


@pytest.mark.parametrize("nM,nN,s", [(96, 96, 2), (48, 48, 4), (24, 40, 2), (136, 136, 2), (12, 12, 2)])
def test_half_spectrum_pack_split_and_hermitian_fold(nM, nN, s):
    """k_o1/k_o2 rewrite of fft2(U1) and the order-2 fold (wst_device.h): two real rows (r and
    r + nM/2, k_o1 step 4) packed as re/im of one complex row, one row FFT, split into the rows'
    half spectra (columns 0..nN/2);
    the column FFT of the half spectrum; the fold reading columns > nN/2 through Hermitian
    symmetry U1hat[kr][kc] = conj(U1hat[-kr][nN-kc])."""
    rng = np.random.default_rng(nM + nN)
    U = rng.random((nM, nN))
    nh = nM // 2
    Z = np.fft.fft(U[:nh] + 1j * U[nh:], axis=1)
    Zm = Z[:, (-np.arange(nN)) % nN]
    hld = nN // 2 + 1
    Xa = (0.5 * (Z + np.conj(Zm)))[:, :hld]
    Xb = (-0.5j * (Z - np.conj(Zm)))[:, :hld]
    H = np.empty((nM, hld), complex)
    H[:nh], H[nh:] = Xa, Xb
    # kernel arithmetic of the split: Xa=((z.x+zm.x)/2,(z.y-zm.y)/2), Xb=((z.y+zm.y)/2,-(z.x-zm.x)/2)
    z, zm = Z[:, :hld], Zm[:, :hld]
    np.testing.assert_allclose(Xa, 0.5 * (z.real + zm.real) + 0.5j * (z.imag - zm.imag), atol=1e-12)
    np.testing.assert_allclose(Xb, 0.5 * (z.imag + zm.imag) - 0.5j * (z.real - zm.real), atol=1e-12)
    H = np.fft.fft(H, axis=0)
    full = np.fft.fft2(U)
    np.testing.assert_allclose(H, full[:, :hld], atol=1e-9)
    psi = rng.random((nM, nN))
    nM2, nN2 = nM // s, nN // s
    ref = (full * psi).reshape(s, nM2, s, nN2).sum(axis=(0, 2))
    got = np.zeros((nM2, nN2), complex)
    for u in range(nM2):
        for v in range(nN2):
            for i in range(s):
                kr_ = u + i * nM2
                for j in range(s):
                    kc = v + j * nN2
                    a = H[kr_, kc] if kc <= nN // 2 else np.conj(H[(nM - kr_) % nM, nN - kc])
                    got[u, v] += a * psi[kr_, kc]
    np.testing.assert_allclose(got, ref, atol=1e-9)
