"""Grid symmetries of the scattering transform (SURVEY.md §4.4's rotation pin), shared by the oracle
test (tests/test_oracle.py) and the GPU test (tests/test_gpu_symmetry.py).

For a square padded plane (pre_pad=True, so no reflect padding enters) of side P with J scales and
Mo x Mo output maps, the kept output points sit at (a + 1) 2^J, a = 0..Mo-1, symmetric about
c = (Mo + 1) 2^J / 2.  The three grid maps below permute the periodic P x P grid about (c, c), so
they commute with the FFTs, the subsampling and the unpad, and act on the filters as

  rot90      y[i, j] = x[j, 2c - i]    theta -> theta + pi/2    l -> (l + L/2) mod L
  flip rows  y[i, j] = x[2c - i, j]    theta -> -theta          l -> (L - 2 - l) mod L
  transpose  y[i, j] = x[j, i]         theta -> pi/2 - theta    l -> (L/2 - 2 - l) mod L

with kymatio's grid theta_l = (int(L - L/2 - 1) - l) pi / L (filter_bank.py; the reference's
compare_wst_coefficients.py:55,67 angle formula) and theta + pi equivalent to theta for |x * psi|
(psi(-u) = conj(psi(u)), x real).  The order-2 indices permute in both theta1 and theta2; each
output map is transformed by the same grid map (rot90: np.rot90(m, 1), flip: flipud, transpose:
m.T), the direction fixed here empirically on the float64 oracle.

What holds exactly: S0, S1 and the order-2 coefficients with j1 = 0 (their filters are level-0
spectra, sampled on the full grid).  The order-2 coefficients with j1 >= 1 use level-j1 crops of
psi_{j2}; kymatio's MASKED crop keeps the negative Nyquist bin and drops the positive one
(periodize_filter_fft), which no rotation or reflection preserves, so they deviate by
~1e-4..1e-3 relative.  A symmetric crop would make them exact: the deviation is asserted to exist,
which pins the masked-crop restatement as well.

What this cannot pin: which array axis the filter's xx coordinate runs along.  Swapping it relabels
l -> (L/2 - 2 - l) mod L, and every permutation above commutes with that relabelling.
"""
import numpy as np

from oracle import kymatio_ref as kr


def geometry(P, J):
    Mo = P // 2 ** J - 2
    return (Mo + 1) * 2 ** J // 2


def grid_ops(P, J, L):
    c = geometry(P, J)
    i = np.arange(P)
    r = (2 * c - i) % P
    return {
        "rot90": (lambda a: np.swapaxes(a[..., :, r], -1, -2),
                  lambda l: (l + L // 2) % L,
                  lambda m: np.rot90(m, 1, axes=(-2, -1))),
        "flip": (lambda a: a[..., r, :],
                 lambda l: (L - 2 - l) % L,
                 lambda m: m[..., ::-1, :]),
        "transpose": (lambda a: np.swapaxes(a, -1, -2),
                      lambda l: (L // 2 - 2 - l) % L,
                      lambda m: np.swapaxes(m, -1, -2)),
    }


def coefficient_permutation(J, L, f):
    """idx[k'] = k such that S(op x)[k'] = mapop(S(x)[idx[k']]) under the orientation map f."""
    K = kr.num_coefficients(J, L)
    idx = np.zeros(K, int)
    for j1 in range(J):
        for l1 in range(L):
            idx[1 + j1 * L + l1] = 1 + j1 * L + f(l1)
    k = 1 + J * L
    for j1 in range(J):
        for l1 in range(L):
            for j2 in range(j1 + 1, J):
                for l2 in range(L):
                    idx[k] = kr.coefficient_index(J, L, j1, f(l1), j2, f(l2))
                    k += 1
    return idx


def exact_mask(J, L):
    """True for the coefficients the grid maps preserve exactly: S0, S1, S2 with j1 = 0."""
    K = kr.num_coefficients(J, L)
    m = np.zeros(K, bool)
    m[:1 + J * L + L * L * (J - 1)] = True
    return m


def symmetry_errors(Sx, Sy, J, L, f, mapop):
    """Per-coefficient error of S(op x) against the permuted, grid-mapped S(x) (leading dims are
    planes), relative to each coefficient's largest value."""
    idx = coefficient_permutation(J, L, f)
    exp = mapop(np.asarray(Sx, np.float64))[..., idx, :, :]
    d = np.abs(np.asarray(Sy, np.float64) - exp)
    K = len(idx)
    num = np.moveaxis(d, -3, 0).reshape(K, -1).max(1)
    den = np.moveaxis(np.abs(exp), -3, 0).reshape(K, -1).max(1)
    return num / np.where(den > 0, den, 1.0)
