"""GPU: SURVEY §4.4's rotation pin on the HIP path (tests/symmetry.py).  For square planes with
even L, S(rot90 x) equals S(x) with the orientation indices permuted by L/2 mod L (S1 in theta1,
S2 in theta1 and theta2) and each map rotated by np.rot90(m, 1); a row flip and a transpose permute
by L-2-l and L/2-2-l.  Bar (written here): the exactly-preserved coefficients (S0, S1, S2 with
j1 = 0) agree GPU-vs-GPU within 2e-5 per coefficient (two fp32 transforms, each within the 1e-5
parity bar); every coefficient of both transforms agrees with the float64 oracle within 1e-5.
Geometries: c2 (64^2, J=4, P=96) and f3 (the reference's 128^2, J=2, P=136)."""
import numpy as np
import pytest

from oracle import kymatio_ref as kr
from parity import TOL, assert_parity
from symmetry import exact_mask, grid_ops, symmetry_errors

from wst_amd.numpy import Scattering2D as NpS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,J", [(64, 4), (128, 2)])
def test_grid_symmetries_on_gpu(M, J):
    L = 8
    s = NpS(J=J, shape=(M, M), L=L, pre_pad=True)
    ref = kr.Scattering2D(J=J, shape=(M, M), L=L, pre_pad=True)
    P = ref.M_padded
    x = (np.random.default_rng(11).integers(0, 256, (3, P, P)) / 255).astype(np.float32)
    Sx = s(x)
    assert_parity(Sx, ref(x.astype(np.float64)), TOL, f"{M} J={J} x", elementwise=False)
    exact = exact_mask(J, L)
    for name, (op, f, mapop) in grid_ops(P, J, L).items():
        y = np.ascontiguousarray(op(x))
        Sy = s(y)
        assert_parity(Sy, ref(y.astype(np.float64)), TOL, f"{M} J={J} {name}", elementwise=False)
        err = symmetry_errors(Sx, Sy, J, L, f, mapop)
        assert err[exact].max() <= 2 * TOL, (name, float(err[exact].max()), int(np.argmax(err * exact)))
