"""Float64 numpy model of the HIP kernels' dataflow (test infrastructure).

It restates what csrc/wst_hip.hip computes -- reflect-index gather, separable spatial low-pass at
the kept points, mean-centred spectra, fold-then-inverse-DFT -- so the CPU suite can check that
those exact rewrites of kymatio's cascade agree with the oracle before any GPU run.
"""
import numpy as np


def reflect_index(i, n):
    if n == 1:
        return 0
    period = 2 * (n - 1)
    t = i % period
    return t if t < n else period - t


def lowpass(U, hM, hN, s, oM, oN):
    rows, cols = U.shape
    S = np.zeros((oM, oN))
    for a in range(oM):
        for c in range(oN):
            im = (s * (a + 1) - np.arange(rows)) % rows
            iq = (s * (c + 1) - np.arange(cols)) % cols
            S[a, c] = hM[im] @ U @ hN[iq]
    return S


def fold(X, psi, nM, nN):
    Y = X * psi
    sM, sN = X.shape[0] // nM, X.shape[1] // nN
    return Y.reshape(sM, nM, sN, nN).sum(axis=(0, 2))


def scatter_model(x, J, L, hM, hN, psi, max_order=2, pre_pad=False):
    """x: (M, N) plane.  hM/hN[r]: spatial taps.  psi[(j, l)][r]: Fourier levels."""
    M, N = x.shape
    PM = ((M + 2 ** J) // 2 ** J + 1) * 2 ** J
    PN = ((N + 2 ** J) // 2 ** J + 1) * 2 ** J
    pt, pl = (PM - M) // 2, (PN - N) // 2
    if pre_pad:
        xp = x
    else:
        xp = np.array([[x[reflect_index(u - pt, M), reflect_index(v - pl, N)] for v in range(PN)]
                       for u in range(PM)])
    oM, oN = (PM >> J) - 2, (PN >> J) - 2
    out = [lowpass(xp, hM[0], hN[0], 2 ** J, oM, oN)]
    Xh = np.fft.fft2(xp - xp.mean())
    S2 = []
    for j1 in range(J):
        for l1 in range(L):
            nM1, nN1 = PM >> j1, PN >> j1
            A = fold(Xh, psi[(j1, l1)][0], nM1, nN1)
            U1 = np.abs(np.fft.ifft2(A) * (nM1 * nN1)) / (PM * PN)
            out.append(lowpass(U1, hM[j1], hN[j1], 2 ** (J - j1), oM, oN))
            if max_order < 2 or j1 >= J - 1:
                continue
            U1h = np.fft.fft2(U1 - U1.mean())
            for j2 in range(j1 + 1, J):
                for l2 in range(L):
                    nM2, nN2 = PM >> j2, PN >> j2
                    B = fold(U1h, psi[(j2, l2)][j1], nM2, nN2)
                    U2 = np.abs(np.fft.ifft2(B) * (nM2 * nN2)) / (nM1 * nN1)
                    S2.append(lowpass(U2, hM[j2], hN[j2], 2 ** (J - j2), oM, oN))
    return np.stack(out + S2)
