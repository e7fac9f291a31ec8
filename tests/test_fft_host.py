"""CPU test of the LDS FFT engine's index math: the library's host emulation of the exact
per-unit device code (csrc/fft_lds.h) against numpy, for every compiled size, both directions,
row- and column-major line layouts, batched arrays and odd padded strides."""
import numpy as np
import pytest

from wst_amd import _lib

COMPILED = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 27, 28, 30,
            32, 34, 36, 40, 44, 48, 52, 54, 56, 60, 64, 68, 72, 80, 88, 96, 104, 108, 112, 120, 128,
            136]
SIZES = COMPILED + [19, 21, 38, 76]    # the last four take the generic-DFT fallback


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("inverse", [False, True])
def test_line_fft_rows_and_cols(n, inverse):
    rng = np.random.default_rng(n)
    nb, rows = 2, 5
    ld = n | 1                            # odd padded row stride, as in the kernels
    bs = rows * ld + 3
    buf = np.zeros(nb * bs, np.complex64)
    x = (rng.standard_normal((nb, rows, n)) + 1j * rng.standard_normal((nb, rows, n))).astype(np.complex64)
    for b in range(nb):
        for r in range(rows):
            buf[b * bs + r * ld: b * bs + r * ld + n] = x[b, r]
    # along rows: nl = rows, ls = ld, es = 1
    for threads in (64, 256):
        y = buf.copy()
        _lib.host_fft_lines(y, n, inverse, nb, bs, rows, ld, 1, threads)
        got = np.stack([np.stack([y[b * bs + r * ld: b * bs + r * ld + n] for r in range(rows)])
                        for b in range(nb)])
        ref = np.fft.ifft(x.astype(np.complex128), axis=-1) * n if inverse else np.fft.fft(x.astype(np.complex128), axis=-1)
        err = np.abs(got - ref).max() / np.abs(ref).max()
        assert err < 3e-6 * max(1.0, np.log2(n)), (n, inverse, threads, err)
    # along columns of an (n x 3) array with row stride 3: nl = 3, ls = 1, es = 3
    cols = 3
    z = (rng.standard_normal((n, cols)) + 1j * rng.standard_normal((n, cols))).astype(np.complex64)
    zb = z.reshape(-1).copy()
    _lib.host_fft_lines(zb, n, inverse, 1, 0, cols, 1, cols, 128, mode=0)
    ref = np.fft.ifft(z.astype(np.complex128), axis=0) * n if inverse else np.fft.fft(z.astype(np.complex128), axis=0)
    err = np.abs(zb.reshape(n, cols) - ref).max() / np.abs(ref).max()
    assert err < 3e-6 * max(1.0, np.log2(n)), (n, inverse, "cols", err)


@pytest.mark.parametrize("n", COMPILED)
@pytest.mark.parametrize("inverse", [False, True])
def test_inplace_digit_reversed_roundtrip(n, inverse):
    """mode 1 (natural -> digit-reversed) and mode 2 (digit-reversed -> natural), as the order-1/2
    kernels chain them: position p of a mode-1 output holds logical bin perm[p]."""
    rng = np.random.default_rng(100 + n)
    rows = 4
    ld = n | 1
    x = (rng.standard_normal((rows, n)) + 1j * rng.standard_normal((rows, n))).astype(np.complex64)
    buf = np.zeros(rows * ld, np.complex64)
    for r in range(rows):
        buf[r * ld: r * ld + n] = x[r]
    y = buf.copy()
    perm = _lib.host_fft_lines(y, n, inverse, 1, 0, rows, ld, 1, 256, mode=1)
    assert sorted(perm.tolist()) == list(range(n))
    got = np.stack([y[r * ld: r * ld + n] for r in range(rows)])
    ref = (np.fft.ifft(x.astype(np.complex128), axis=-1) * n if inverse
           else np.fft.fft(x.astype(np.complex128), axis=-1))
    tol = 3e-6 * max(1.0, np.log2(n))
    assert np.abs(got - ref[:, perm]).max() / np.abs(ref).max() < tol
    # mode 2 on digit-reversed input returns natural order
    z = np.zeros(rows * ld, np.complex64)
    for r in range(rows):
        z[r * ld: r * ld + n] = x[r][perm]
    _lib.host_fft_lines(z, n, inverse, 1, 0, rows, ld, 1, 256, mode=2)
    got2 = np.stack([z[r * ld: r * ld + n] for r in range(rows)])
    assert np.abs(got2 - ref).max() / np.abs(ref).max() < tol


@pytest.mark.parametrize("n", [n for n in COMPILED if n > 16 and n not in (17,)])
@pytest.mark.parametrize("inverse", [False, True])
def test_rd_from_global_equals_inplace(n, inverse):
    """mode 3 (k_o2's spectrum column transform: G whose first stage reads the workspace rows
    instead of an LDS copy, csrc/fft_lds.h fft_lines_rd_from) is bitwise mode 2 on the same input,
    along columns of a half-spectrum-shaped array (nl = hld columns, ls = 1, es = hld)."""
    rng = np.random.default_rng(200 + n)
    hld = n // 2 + 1
    a = (rng.standard_normal(n * hld) + 1j * rng.standard_normal(n * hld)).astype(np.complex64)
    ref, got = a.copy(), a.copy()
    _lib.host_fft_lines(ref, n, inverse, 1, 0, hld, 1, hld, 256, mode=2)
    _lib.host_fft_lines(got, n, inverse, 1, 0, hld, 1, hld, 256, mode=3)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), n


@pytest.mark.parametrize("nn,rs", [(48, 8)])
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_row_split_column_remap(nn, rs, inverse):
    """The S2 pass of the 48^2 order-2 paths (csrc/wst_device.h cols_modlp RS) walks the tap matrix
    GN in the split_n2 digit-reversed order and reads each logical column's partial from its place
    in the rows' order (split (nn / rs) x rs, fused_row_n2): the remap must land every GN row on the
    physical column that holds the same logical column.  Both sides come from the library: the
    split_n2 order from mode 1, the rows' order from mode 4 (the transform with the fused rows'
    split, LineFFT<48, true, 8>), whose output is also checked to be that permutation of the DFT."""
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(nn) + 1j * rng.standard_normal(nn)).astype(np.complex64)
    perm_default = _lib.host_fft_lines(x.copy(), nn, inverse, 1, 0, 1, nn, 1, 64, mode=1)
    y = x.copy()
    perm_rows = _lib.host_fft_lines(y, nn, inverse, 1, 0, 1, nn, 1, 64, mode=4)
    ref = np.fft.ifft(x.astype(np.complex128)) * nn if inverse else np.fft.fft(x.astype(np.complex128))
    assert np.abs(y - ref[perm_rows]).max() / np.abs(ref).max() < 3e-6 * np.log2(nn)
    n2d = next(d for d in range(int(nn ** 0.5), 0, -1) if nn % d == 0)
    n1d, n1r = nn // n2d, nn // rs
    seen = set()
    for q in range(nn):
        lg = q // n2d + n1d * (q % n2d)
        assert lg == perm_default[q]
        qr = rs * (lg % n1r) + lg // n1r               # the kernel's remap (cols_modlp RS)
        assert perm_rows[qr] == lg                     # the rows' transform holds lg there
        seen.add(qr)
    assert seen == set(range(nn))
