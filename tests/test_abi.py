"""CPU tests of the C-ABI library: it loads, exports every symbol include/wst_hip.h declares,
and its host-side float64 filter construction matches the oracle (no GPU compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import kymatio_ref as kr
from wst_amd import _lib

HEADER = os.path.join(ROOT, "include", "wst_hip.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(wst_\w+)\s*\(", src, re.M)))


def test_library_loads_and_exports_header_symbols():
    lib = _lib.load()
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTS), syms
    for s in syms:
        assert getattr(lib, s) is not None
        assert ctypes.cast(getattr(lib, s), ctypes.c_void_p).value
    assert lib.wst_abi_version() == _lib.ABI_VERSION


def test_invalid_configs_rejected_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.wst_plan_create(8, 8, 4, 8, 2, 0, ctypes.byref(h)) == _lib.WST_ERR_INVALID
    assert "2^J" in _lib.last_error()
    assert lib.wst_plan_create(64, 64, 2, 8, 3, 0, ctypes.byref(h)) == _lib.WST_ERR_INVALID
    assert lib.wst_plan_create(64, 64, 0, 8, 2, 0, ctypes.byref(h)) == _lib.WST_ERR_INVALID
    assert lib.wst_plan_create(64, 64, 2, 8, 2, 0, None) == _lib.WST_ERR_INVALID
    assert lib.wst_output_shape(None, None, None, None) == _lib.WST_ERR_INVALID
    assert lib.wst_plan_destroy(None) == _lib.WST_OK


@pytest.mark.parametrize("M,N,J,L", [(64, 64, 2, 8), (64, 64, 4, 8), (32, 32, 3, 6), (40, 56, 2, 5)])
def test_host_filter_bank_matches_oracle(M, N, J, L):
    PM, PN = kr.compute_padding(M, N, J)
    fb = kr.filter_bank(PM, PN, J, L)
    for p in fb["psi"]:
        for r, lev in enumerate(p["levels"]):
            h = _lib.host_filter(M, N, J, L, 0, p["j"], p["theta"], r, lev.size).reshape(lev.shape)
            assert np.abs(h - lev).max() <= 1e-13 * np.abs(lev).max()
    for r, lev in enumerate(fb["phi"]["levels"]):
        h = _lib.host_filter(M, N, J, L, 1, 0, 0, r, lev.size).reshape(lev.shape)
        assert np.abs(h - lev).max() <= 1e-13 * np.abs(lev).max()
        # the separable spatial low-pass the kernels use: outer(hM, hN) == ifft2(phi level)
        hm = _lib.host_filter(M, N, J, L, 2, 0, 0, r, PM >> r)
        hn = _lib.host_filter(M, N, J, L, 3, 0, 0, r, PN >> r)
        sp = np.fft.ifft2(lev)
        assert np.abs(sp.imag).max() < 1e-15
        assert np.abs(np.outer(hm, hn) - sp.real).max() <= 1e-13 * np.abs(sp.real).max()


def test_host_filter_errors():
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(64, 64, 2, 8, 0, 5, 0, 0, 72 * 72)       # j out of range
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(64, 64, 2, 8, 0, 0, 0, 1, 36 * 36)       # psi_0 has 1 level at J=2
    with pytest.raises(_lib.WSTError):
        _lib.host_filter(64, 64, 2, 8, 1, 0, 0, 0, 10)            # buffer too small
