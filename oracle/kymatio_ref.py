"""CPU float64 restatement of kymatio 0.3.0 ``Scattering2D`` -- TEST INFRASTRUCTURE ONLY.

This module is the parity *oracle*.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed CPU
baseline.  The product path (``wst_amd``) never imports it: it runs the HIP library or raises.

Provenance
----------
The reference repository calls ``kymatio==0.3.0`` (``requirements.txt:18``) from
``src/training/train_and_save_model.py:46,359,368`` (numpy frontend),
``src/inference/inference.py:39,242,254`` (torch frontend) and
``src/visualization/compare_wst_coefficients.py:15,37`` (``frontend='numpy'``).
kymatio is a third-party dependency that is *not* vendored under /root/reference and is not
installed in this image; executing the reference's own modules was denied.
This file therefore restates kymatio 0.3.0's published algorithm:

* ``compute_padding``        <- [kymatio 0.3.0] scattering2d/utils.py
* ``gabor_2d``/``morlet_2d`` <- [kymatio 0.3.0] scattering2d/filter_bank.py
* ``periodize_filter_fft``   <- [kymatio 0.3.0] scattering2d/filter_bank.py (masked crop, A.3)
* ``filter_bank``            <- [kymatio 0.3.0] scattering2d/filter_bank.py
* ``pad``/``unpad``/``subsample_fourier``/``cdgmm``/``modulus``/FFTs
                             <- [kymatio 0.3.0] scattering2d/backend/numpy_backend.py
* ``scattering2d``           <- [kymatio 0.3.0] scattering2d/core/scattering2d.py
* ``Scattering2D``           <- [kymatio 0.3.0] frontend/base_frontend.py + numpy_frontend.py
* ``extract_wst_features``   <- reference ``src/training/train_and_save_model.py:346-378``

Parity status: *pinned by analytic known answers and layout contracts only* -- no kymatio
golden vector exists in the reference or in this container.  The
golden fixtures under ``tests/golden/`` are generated from this restatement by
``tests/golden/make_golden.py``.

Arithmetic: float64 everywhere (kymatio's numpy backend promotes to complex128 at the first
filter multiply; its very first FFT of a float32 input may run in complex64 -- a ~1e-7
relative difference, far below the 1e-5 parity tolerance).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.fft

__all__ = [
    "compute_padding", "gabor_2d", "morlet_2d", "periodize_filter_fft", "filter_bank",
    "reflect_pad", "unpad", "subsample_fourier", "scattering2d", "Scattering2D",
    "num_coefficients", "extract_wst_features", "extract_wst_features_interleaved",
    "coefficient_index", "FilterConvention", "KYMATIO_0_3_0",
]


# --------------------------------------------------------------------------------------
# Version-dependent constants of kymatio's filter construction, in ONE place
# --------------------------------------------------------------------------------------
@dataclass(frozen=True)
class FilterConvention:
    """The constants of kymatio's ``gabor_2d`` that are recalled from upstream 0.3.0 rather than
    read from its source (kymatio is absent: SURVEY.md §8(c)).  The HIP library takes the same
    struct as its plan parameter (``wst_filter_convention``, include/wst_hip.h; defaults in
    csrc/filter_bank.h ``kKymatio030``), so oracle and product switch together.

    norm_pi         "pi" of the normaliser 2*pi*sigma^2/slant.  Upstream writes the literal
                    3.1415 (phi_hat(0) = pi/3.1415).  Every S0 / S1 / S2 scales by
                    (3.1415/norm_pi)^(1, 2, 3): ~3e-5 / 6e-5 / 9e-5 relative for np.pi.
    periodize_half  the periodisation grid ex, ey in [-h, h] (5x5 copies for h = 2).
    gabor_dtype     accumulator of gabor_2d (complex128; complex64 in versions that allocate
                    ``np.zeros((M, N), np.complex64)``).  Oracle-only switch: the device filters
                    are float32 either way (tests/test_convention.py measures its effect).
    rot_dtype       dtype of gabor_2d's rotation matrices R, R_inv (float64; versions that write
                    ``np.array(..., np.float32)`` round cos/sin of theta to float32 in the
                    envelope's curvature, not in the modulation).  Shared with the library
                    (wst_filter_convention flags bit 0)."""
    norm_pi: float = 3.1415
    periodize_half: int = 2
    gabor_dtype: type = np.complex128
    rot_dtype: type = np.float64


KYMATIO_0_3_0 = FilterConvention()


# --------------------------------------------------------------------------------------
# A.1 sizes
# --------------------------------------------------------------------------------------
def compute_padding(M: int, N: int, J: int) -> tuple[int, int]:
    """[kymatio 0.3.0] scattering2d/utils.py ``compute_padding``."""
    M_padded = ((M + 2 ** J) // 2 ** J + 1) * 2 ** J
    N_padded = ((N + 2 ** J) // 2 ** J + 1) * 2 ** J
    return M_padded, N_padded


def num_coefficients(J: int, L: int, max_order: int = 2) -> int:
    """K = 1 + J*L (+ L^2*J*(J-1)/2 at order 2).  Layout pin:
    reference ``src/visualization/compare_wst_coefficients.py:44-52``."""
    K = 1 + J * L
    if max_order >= 2:
        K += L * L * J * (J - 1) // 2
    return K


def coefficient_index(J: int, L: int, j1: int, l1: int, j2: int | None = None,
                      l2: int | None = None) -> int:
    """Flat coefficient index in kymatio order: [S0; S1 (j1-major, l1-minor);
    S2 (n1 in psi order, n2 in psi order with j2 > j1)]."""
    if j2 is None:
        return 1 + j1 * L + l1
    k = 1 + J * L
    for jj1 in range(J):
        for ll1 in range(L):
            for jj2 in range(jj1 + 1, J):
                for ll2 in range(L):
                    if (jj1, ll1, jj2, ll2) == (j1, l1, j2, l2):
                        return k
                    k += 1
    raise ValueError("invalid (j1, l1, j2, l2)")


# --------------------------------------------------------------------------------------
# A.2 filters
# --------------------------------------------------------------------------------------
def gabor_2d(M, N, sigma, theta, xi, slant=1.0, offset=0, conv=KYMATIO_0_3_0):
    """[kymatio 0.3.0] filter_bank.py ``gabor_2d``: periodised (5x5 copies) Gabor in space.
    ``xx`` runs along axis 0 on the asymmetric grid [ex*M, ex*M + M).  ``conv`` holds the
    recalled constants (FilterConvention)."""
    gab = np.zeros((M, N), conv.gabor_dtype)
    R = np.array([[np.cos(theta), -np.sin(theta)], [np.sin(theta), np.cos(theta)]], conv.rot_dtype)
    R_inv = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]], conv.rot_dtype)
    D = np.array([[1, 0], [0, slant * slant]])
    curv = np.dot(R, np.dot(D, R_inv)) / (2 * sigma * sigma)
    h = conv.periodize_half
    for ex in range(-h, h + 1):
        for ey in range(-h, h + 1):
            xx, yy = np.mgrid[offset + ex * M:offset + M + ex * M,
                              offset + ey * N:offset + N + ey * N]
            arg = -(curv[0, 0] * xx * xx + (curv[0, 1] + curv[1, 0]) * xx * yy
                    + curv[1, 1] * yy * yy) \
                + 1.j * (xx * np.cos(theta) * xi + yy * np.sin(theta) * xi)
            gab += np.exp(arg)
    norm_factor = 2 * conv.norm_pi * sigma * sigma / slant   # literal 3.1415 upstream
    gab /= norm_factor
    return gab


def morlet_2d(M, N, sigma, theta, xi, slant=0.5, offset=0, conv=KYMATIO_0_3_0):
    """[kymatio 0.3.0] filter_bank.py ``morlet_2d`` = gabor(xi) - K * gabor(0), zero mean."""
    wv = gabor_2d(M, N, sigma, theta, xi, slant, offset, conv)
    wv_modulus = gabor_2d(M, N, sigma, theta, 0, slant, offset, conv)
    K = np.sum(wv) / np.sum(wv_modulus)
    return wv - K * wv_modulus


def periodize_filter_fft(x, res):
    """[kymatio 0.3.0] filter_bank.py ``periodize_filter_fft``: MASKED crop.

    Zero rows/cols [M*2^-(res+1), M*2^-(res+1) + M*(1-2^-res)), then sum the 2^res x 2^res
    alias blocks.  Net effect: a crop of bins [-M/2^(res+1), M/2^(res+1)) (negative Nyquist
    kept, positive Nyquist dropped).  The alias sum is the vectorised form of upstream's
    four nested loops ``crop[k,l] += x[k + i*M/2^res, l + j*N/2^res]``."""
    M, N = x.shape
    mask = np.ones(x.shape, np.float32)
    len_x = int(M * (1 - 2 ** (-res)))
    start_x = int(M * 2 ** (-res - 1))
    len_y = int(N * (1 - 2 ** (-res)))
    start_y = int(N * 2 ** (-res - 1))
    mask[start_x:start_x + len_x, :] = 0
    mask[:, start_y:start_y + len_y] = 0
    x = np.multiply(x, mask)
    s = 2 ** res
    Ms, Ns = int(M / s), int(N / s)
    return x.reshape(s, Ms, s, Ns).sum(axis=(0, 2)).astype(x.dtype)


def periodize_filter_fft_loops(x, res):
    """Literal four-loop form of the crop (small sizes only; used to pin the vectorised one)."""
    M, N = x.shape
    crop = np.zeros((M // 2 ** res, N // 2 ** res), x.dtype)
    mask = np.ones(x.shape, np.float32)
    len_x = int(M * (1 - 2 ** (-res)))
    start_x = int(M * 2 ** (-res - 1))
    len_y = int(N * (1 - 2 ** (-res)))
    start_y = int(N * 2 ** (-res - 1))
    mask[start_x:start_x + len_x, :] = 0
    mask[:, start_y:start_y + len_y] = 0
    x = np.multiply(x, mask)
    for k in range(int(M / 2 ** res)):
        for l in range(int(N / 2 ** res)):
            for i in range(int(2 ** res)):
                for j in range(int(2 ** res)):
                    crop[k, l] += x[k + i * int(M / 2 ** res), l + j * int(N / 2 ** res)]
    return crop


def filter_bank(M, N, J, L=8, conv=KYMATIO_0_3_0):
    """[kymatio 0.3.0] filter_bank.py ``filter_bank`` on the PADDED grid (M, N).

    psi_{j,l}: sigma=0.8*2^j, theta=(int(L-L/2-1)-l)*pi/L, xi=3pi/(4*2^j), slant=4/L,
    Fourier levels r < min(j+1, max(J-1,1)).  phi: gabor(sigma=0.8*2^(J-1), 0, 0), levels r<J.
    Spectra are Re(fft2(.)) (imaginary part ~1e-16)."""
    filters = {"psi": []}
    for j in range(J):
        for theta in range(L):
            psi = {"levels": [], "j": j, "theta": theta}
            psi_signal = morlet_2d(M, N, 0.8 * 2 ** j, (int(L - L / 2 - 1) - theta) * np.pi / L,
                                   3.0 / 4.0 * np.pi / 2 ** j, 4.0 / L, conv=conv)
            psi_signal_fourier = np.real(scipy.fft.fft2(psi_signal))
            for res in range(min(j + 1, max(J - 1, 1))):
                psi["levels"].append(periodize_filter_fft(psi_signal_fourier, res))
            filters["psi"].append(psi)
    phi_signal = gabor_2d(M, N, 0.8 * 2 ** (J - 1), 0, 0, conv=conv)
    phi_signal_fourier = np.real(scipy.fft.fft2(phi_signal))
    filters["phi"] = {"levels": [], "j": J}
    for res in range(J):
        filters["phi"]["levels"].append(periodize_filter_fft(phi_signal_fourier, res))
    return filters


# --------------------------------------------------------------------------------------
# backend primitives (numpy backend)
# --------------------------------------------------------------------------------------
def reflect_pad(x, pad_size):
    """[kymatio 0.3.0] numpy_backend ``Pad``: np.pad mode='reflect' (no edge repeat).
    pad_size = [top, bottom, left, right]."""
    return np.pad(x, ((0, 0), (pad_size[0], pad_size[1]), (pad_size[2], pad_size[3])),
                  mode="reflect")


def unpad(x):
    """[kymatio 0.3.0] numpy_backend ``unpad``: crop one sample on every side."""
    return x[..., 1:-1, 1:-1]


def subsample_fourier(x, k):
    """[kymatio 0.3.0] numpy_backend ``subsample_fourier``: mean over the k x k alias blocks
    (== spatial decimation by k after the inverse FFT)."""
    y = x.reshape(-1, k, x.shape[-2] // k, k, x.shape[-1] // k)
    return y.mean(axis=(-4, -2))


def cdgmm(A, B):
    return A * B


def modulus(x):
    return np.abs(x)


def _fft2(x):
    return scipy.fft.fft2(x, axes=(-2, -1))


def _ifft2(x):
    return scipy.fft.ifft2(x, axes=(-2, -1))


# --------------------------------------------------------------------------------------
# A.4 cascade
# --------------------------------------------------------------------------------------
def scattering2d(x, pad, J, L, phi, psi, max_order, out_type="array"):
    """[kymatio 0.3.0] core/scattering2d.py ``scattering2d`` on a (B, M, N) float64 stack."""
    out_S_0, out_S_1, out_S_2 = [], [], []
    U_r = pad(x)
    U_0_c = _fft2(U_r)

    U_1_c = cdgmm(U_0_c, phi["levels"][0])
    U_1_c = subsample_fourier(U_1_c, k=2 ** J)
    S_0 = unpad(_ifft2(U_1_c).real)
    out_S_0.append({"coef": S_0, "j": (), "theta": ()})

    for n1 in range(len(psi)):
        j1 = psi[n1]["j"]
        theta1 = psi[n1]["theta"]
        U_1_c = cdgmm(U_0_c, psi[n1]["levels"][0])
        if j1 > 0:
            U_1_c = subsample_fourier(U_1_c, k=2 ** j1)
        U_1_c = _ifft2(U_1_c)
        U_1_c = modulus(U_1_c)
        U_1_c = _fft2(U_1_c)

        S_1_c = cdgmm(U_1_c, phi["levels"][j1])
        S_1_c = subsample_fourier(S_1_c, k=2 ** (J - j1))
        S_1_r = unpad(_ifft2(S_1_c).real)
        out_S_1.append({"coef": S_1_r, "j": (j1,), "theta": (theta1,)})

        if max_order < 2:
            continue
        for n2 in range(len(psi)):
            j2 = psi[n2]["j"]
            theta2 = psi[n2]["theta"]
            if j2 <= j1:
                continue
            U_2_c = cdgmm(U_1_c, psi[n2]["levels"][j1])
            U_2_c = subsample_fourier(U_2_c, k=2 ** (j2 - j1))
            U_2_c = _ifft2(U_2_c)
            U_2_c = modulus(U_2_c)
            U_2_c = _fft2(U_2_c)

            S_2_c = cdgmm(U_2_c, phi["levels"][j2])
            S_2_c = subsample_fourier(S_2_c, k=2 ** (J - j2))
            S_2_r = unpad(_ifft2(S_2_c).real)
            out_S_2.append({"coef": S_2_r, "j": (j1, j2), "theta": (theta1, theta2)})

    out_S = out_S_0 + out_S_1 + out_S_2
    if out_type == "array":
        return np.stack([s["coef"] for s in out_S], axis=-3)
    return out_S


class Scattering2D:
    """Oracle mirror of kymatio 0.3.0 numpy ``Scattering2D`` (same checks, float64 math)."""

    def __init__(self, J, shape, L=8, max_order=2, pre_pad=False, backend=None,
                 out_type="array", convention=KYMATIO_0_3_0):
        self.J, self.L, self.max_order, self.pre_pad = J, L, max_order, pre_pad
        self.out_type = out_type
        self.shape = tuple(shape)
        M, N = self.shape
        self.M, self.N = M, N
        if 2 ** J > M or 2 ** J > N:
            raise RuntimeError("The smallest dimension should be larger than 2^J.")
        self.M_padded, self.N_padded = compute_padding(M, N, J)
        self.pad_size = [(self.M_padded - M) // 2, (self.M_padded - M + 1) // 2,
                         (self.N_padded - N) // 2, (self.N_padded - N + 1) // 2]
        filters = filter_bank(self.M_padded, self.N_padded, J, L, convention)
        self.phi, self.psi = filters["phi"], filters["psi"]

    def _pad(self, x):
        return x if self.pre_pad else reflect_pad(x, self.pad_size)

    def scattering(self, input):
        if not isinstance(input, np.ndarray):
            raise TypeError("The input should be a NumPy array.")
        if input.ndim < 2:
            raise RuntimeError("Input array must have at least two dimensions.")
        if (input.shape[-1] != self.N or input.shape[-2] != self.M) and not self.pre_pad:
            raise RuntimeError("NumPy array must be of spatial size (%i,%i)." % (self.M, self.N))
        if (input.shape[-1] != self.N_padded or input.shape[-2] != self.M_padded) and self.pre_pad:
            raise RuntimeError("Padded array must be of spatial size (%i,%i)."
                               % (self.M_padded, self.N_padded))
        if self.out_type not in ("array", "list"):
            raise RuntimeError("The out_type must be one of 'array' or 'list'.")
        batch_shape = input.shape[:-2]
        x = np.asarray(input, np.float64).reshape((-1,) + input.shape[-2:])
        S = scattering2d(x, self._pad, self.J, self.L, self.phi, self.psi, self.max_order,
                         self.out_type)
        if self.out_type == "array":
            return S.reshape(batch_shape + S.shape[-3:])
        for s in S:
            s["coef"] = s["coef"].reshape(batch_shape + s["coef"].shape[-2:])
        return S

    __call__ = scattering


# --------------------------------------------------------------------------------------
# reference caller (L2): feature layouts
# --------------------------------------------------------------------------------------
def extract_wst_features(rgb_image, J=2, L=8, scattering=None):
    """Reference ``train_and_save_model.py:346-378``: per channel [mean(K) | std(K)]
    (population std, ddof=0), channels concatenated -> (C*2*K,) float64."""
    C, H, W = rgb_image.shape
    if scattering is None:
        scattering = Scattering2D(J=J, L=L, shape=(H, W))
    feats = []
    for c in range(C):
        coeffs = scattering(rgb_image[c])
        feats.extend(np.concatenate([np.mean(coeffs, axis=(-2, -1)),
                                     np.std(coeffs, axis=(-2, -1))]))
    return np.array(feats)


def extract_wst_features_interleaved(rgb_image, J=2, L=8, scattering=None):
    """Reference ``inference.py:237-270``: per channel interleaved [m_0, s_0, m_1, s_1, ...]."""
    C, H, W = rgb_image.shape
    if scattering is None:
        scattering = Scattering2D(J=J, L=L, shape=(H, W))
    out = []
    for c in range(C):
        coeffs = scattering(rgb_image[c])
        f = np.zeros(2 * coeffs.shape[0])
        f[0::2] = coeffs.reshape(coeffs.shape[0], -1).mean(axis=1)
        f[1::2] = coeffs.reshape(coeffs.shape[0], -1).std(axis=1)
        out.append(f)
    return np.concatenate(out)
