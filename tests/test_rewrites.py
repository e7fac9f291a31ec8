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
