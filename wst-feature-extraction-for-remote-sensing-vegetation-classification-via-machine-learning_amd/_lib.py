"""ctypes binding of the in-tree C-ABI library ``libwst_hip.so`` (include/wst_hip.h).

There is no CPU fallback: if the library is missing, or no ROCm GPU is visible, every compute
entry point raises ``RuntimeError``.  Only the host-side filter inspection
(``host_filter``) runs without a GPU (it is pure C++ float64 code inside the same library).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libwst_hip.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)

WST_OK, WST_ERR_INVALID, WST_ERR_UNSUPPORTED, WST_ERR_HIP, WST_ERR_NOMEM = 0, 1, 2, 3, 4
ABI_VERSION = 2

# every symbol include/wst_hip.h declares
EXPORTS = (
    "wst_abi_version", "wst_last_error", "wst_default_convention", "wst_plan_create",
    "wst_plan_create_ex", "wst_plan_destroy",
    "wst_output_shape", "wst_padded_shape", "wst_workspace_bytes", "wst_preferred_batch",
    "wst_internal_workspaces", "wst_plan_staging",
    "wst_forward",
    "wst_forward_profiled", "wst_host_filter", "wst_host_filter_ex", "wst_host_fft_lines",
    "wst_salt_pepper_counts", "wst_noise_apply", "wst_noise_generate", "wst_advanced_stats",
    "wst_patch_generate", "wst_u8_to_chw", "wst_probe_copy", "wst_probe_fma",
    "wst_aux_last_error", "wst_plan_variants", "wst_describe_variants", "wst_plan_trace",
    "wst_plan_read_trace",
)

_lib = None
_lock = threading.Lock()


def use_library(name: str) -> None:
    """Development tools only (tools/kernel_ms.py, tools/ablate.py): load the variant build
    `name` (a file in the package directory, e.g. a WST_DIAG build) instead of libwst_hip.so.
    Must run before the first load(); the product path never calls it, and no environment
    variable selects a library."""
    global LIB_NAME, LIB_PATH
    if _lib is not None:
        raise RuntimeError(f"{LIB_NAME} is already loaded")
    LIB_NAME = os.path.basename(name)
    LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)


class Convention(ctypes.Structure):
    """``wst_filter_convention`` (include/wst_hip.h): the recalled kymatio constants, mirrored by
    ``oracle.kymatio_ref.FilterConvention``.  Defaults = kymatio 0.3.0 (3.1415, 5x5 grid)."""
    _fields_ = [("norm_pi", ctypes.c_double), ("periodize_half", ctypes.c_int),
                ("flags", ctypes.c_int)]

    def __init__(self, norm_pi=3.1415, periodize_half=2, rot_f32=False, flags=None):
        super().__init__(float(norm_pi), int(periodize_half),
                         int(flags) if flags is not None else (1 if rot_f32 else 0))


def _conv_ptr(convention):
    if convention is None:
        return None
    if not isinstance(convention, Convention):   # anything with the two fields (oracle's class)
        import numpy as _np
        rot32 = getattr(convention, "rot_dtype", _np.float64) == _np.float32
        convention = Convention(convention.norm_pi, convention.periodize_half, rot_f32=rot32)
    return ctypes.byref(convention)


class WSTError(RuntimeError):
    """Raised for a non-zero status from the C ABI."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


TRACE_LIB_NAME = "libwst_hip_trace.so"   # the same sources with -DWST_TRACE (tests only)
_trace_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and type the library.  Raises RuntimeError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        _lib = _open(LIB_PATH, LIB_NAME)
        return _lib


def load_trace() -> ctypes.CDLL:
    """The variant-trace build (tests/test_gpu_variants.py): kernels that record which body and
    level branches they ran (wst_plan_trace); the product library carries no trace code."""
    global _trace_lib
    with _lock:
        if _trace_lib is None:
            _trace_lib = _open(os.path.join(PKG_DIR, TRACE_LIB_NAME), TRACE_LIB_NAME)
        return _trace_lib


def _open(path, name) -> ctypes.CDLL:
    """Open and type one build of the library."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"{name} not found at {path}: the HIP extension is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C <pkg>/csrc`)")
    lib = ctypes.CDLL(path)
    c_int, c_i64, c_vp, c_sz = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t
    lib.wst_abi_version.restype = c_int
    lib.wst_abi_version.argtypes = []
    lib.wst_last_error.restype = ctypes.c_char_p
    lib.wst_last_error.argtypes = []
    lib.wst_plan_create.restype = c_int
    lib.wst_plan_create.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int,
                                    ctypes.POINTER(c_vp)]
    conv_p = ctypes.POINTER(Convention)
    lib.wst_default_convention.restype = c_int
    lib.wst_default_convention.argtypes = [conv_p]
    lib.wst_plan_create_ex.restype = c_int
    lib.wst_plan_create_ex.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int, conv_p,
                                       ctypes.POINTER(c_vp)]
    lib.wst_host_filter_ex.restype = c_int
    lib.wst_host_filter_ex.argtypes = [c_int] * 8 + [conv_p, ctypes.POINTER(ctypes.c_double),
                                                     c_i64]
    lib.wst_plan_destroy.restype = c_int
    lib.wst_plan_destroy.argtypes = [c_vp]
    lib.wst_output_shape.restype = c_int
    lib.wst_output_shape.argtypes = [c_vp] + [ctypes.POINTER(c_int)] * 3
    lib.wst_padded_shape.restype = c_int
    lib.wst_padded_shape.argtypes = [c_vp] + [ctypes.POINTER(c_int)] * 2
    lib.wst_workspace_bytes.restype = c_int
    lib.wst_workspace_bytes.argtypes = [c_vp, c_i64, ctypes.POINTER(c_sz)]
    u8p, f64p, i32p = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p
    lib.wst_salt_pepper_counts.restype = c_int
    lib.wst_salt_pepper_counts.argtypes = [c_int, c_int, c_int, ctypes.c_double,
                                           ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]
    lib.wst_noise_apply.restype = c_int
    lib.wst_noise_apply.argtypes = [c_int, ctypes.c_double, u8p, c_i64, c_int, c_int, c_int,
                                    f64p, i32p, i32p, c_int, c_vp, c_vp]
    lib.wst_noise_generate.restype = c_int
    lib.wst_noise_generate.argtypes = [c_int, ctypes.c_double, u8p, c_i64, c_int, c_int, c_int,
                                       ctypes.c_uint64, c_int, c_vp, c_vp]
    lib.wst_advanced_stats.restype = c_int
    lib.wst_advanced_stats.argtypes = [c_vp, c_i64, c_int, c_int, c_vp, c_vp]
    lib.wst_patch_generate.restype = c_int
    lib.wst_patch_generate.argtypes = [ctypes.c_uint64, c_i64, c_i64, c_int, c_int, c_int, c_int,
                                       c_vp, c_vp]
    lib.wst_u8_to_chw.restype = c_int
    lib.wst_u8_to_chw.argtypes = [c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp]
    lib.wst_probe_copy.restype = c_int
    lib.wst_probe_copy.argtypes = [c_vp, c_vp, c_sz, c_vp]
    lib.wst_probe_fma.restype = c_int
    lib.wst_probe_fma.argtypes = [c_vp, c_i64, c_int, c_vp]
    lib.wst_aux_last_error.restype = ctypes.c_char_p
    lib.wst_aux_last_error.argtypes = []
    lib.wst_preferred_batch.restype = c_int
    lib.wst_preferred_batch.argtypes = [c_vp, ctypes.POINTER(c_i64)]
    lib.wst_plan_staging.restype = c_int
    lib.wst_plan_staging.argtypes = [c_vp] + [ctypes.POINTER(c_int)] * 3
    lib.wst_internal_workspaces.restype = c_int
    lib.wst_internal_workspaces.argtypes = [c_vp, ctypes.POINTER(c_int), ctypes.POINTER(c_sz)]
    lib.wst_forward.restype = c_int
    lib.wst_forward.argtypes = [c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_sz, c_vp]
    lib.wst_forward_profiled.restype = c_int
    lib.wst_forward_profiled.argtypes = [c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_sz, c_vp,
                                         ctypes.POINTER(ctypes.c_float), c_int]
    lib.wst_host_filter.restype = c_int
    lib.wst_host_filter.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    ctypes.POINTER(ctypes.c_double), c_i64]
    lib.wst_host_fft_lines.restype = c_int
    lib.wst_host_fft_lines.argtypes = [c_int, c_int, c_int, c_vp] + [c_int] * 6 + [c_vp]
    i64p = ctypes.POINTER(c_i64)
    # (an older A/B build chosen by use_library may lack the introspection entry points;
    # tests/test_abi.py checks the product library exports all of EXPORTS)
    if hasattr(lib, "wst_plan_variants"):
        lib.wst_plan_variants.restype = c_int
        lib.wst_plan_variants.argtypes = [c_vp, c_vp, c_i64, i64p]
        lib.wst_describe_variants.restype = c_int
        lib.wst_describe_variants.argtypes = [c_int] * 5 + [c_vp, c_i64, i64p]
        lib.wst_plan_trace.restype = c_int
        lib.wst_plan_trace.argtypes = [c_vp, c_int]
        lib.wst_plan_read_trace.restype = c_int
        lib.wst_plan_read_trace.argtypes = [c_vp, c_vp, c_i64, i64p]
    v = lib.wst_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"{name} ABI version {v} != expected {ABI_VERSION}; rebuild it")
    return lib


def last_error() -> str:
    return load().wst_last_error().decode(errors="replace")


def aux_last_error() -> str:
    return (load().wst_aux_last_error() or b"").decode()


def check_aux(code: int) -> None:
    """Status check of the wst_noise_* / wst_advanced_stats entry points."""
    if code != WST_OK:
        raise WSTError(code, aux_last_error() or f"wst status {code}")


def check(code: int) -> None:
    if code != WST_OK:
        raise WSTError(code, last_error() or f"wst status {code}")


def host_filter(M, N, J, L, kind, j, l, r, size, convention=None) -> np.ndarray:
    """Host float64 filter from the library's own construction (no GPU needed)."""
    out = np.zeros(size, np.float64)
    check(load().wst_host_filter_ex(M, N, J, L, kind, j, l, r, _conv_ptr(convention),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), size))
    return out


def describe_variants(M, N, J, L, max_order=2) -> np.ndarray:
    """Trace words (sites x 12, int32) one chunk of a plan for this geometry launches, from the
    library's host mirror of the kernels' dispatch; no GPU needed (wst_describe_variants)."""
    lib = load()
    n = ctypes.c_int64()
    check(lib.wst_describe_variants(int(M), int(N), int(J), int(L), int(max_order), None, 0, ctypes.byref(n)))
    out = np.zeros(max(n.value, 1), np.int32)
    check(lib.wst_describe_variants(int(M), int(N), int(J), int(L), int(max_order), out.ctypes.data,
                                    out.size, ctypes.byref(n)))
    return out[:n.value].reshape(-1, 12)


def default_convention() -> Convention:
    c = Convention()
    check(load().wst_default_convention(ctypes.byref(c)))
    return c


def host_fft_lines(data: np.ndarray, n, inverse, nb, bs, nl, ls, es, threads=256, mode=0):
    """In-place host emulation of the device line FFT on a complex64 buffer (test hook).
    mode 0 natural->natural, 1 natural->digit-reversed, 2 digit-reversed->natural, 3 = mode 2 with
    the first stage reading a copy of the input (k_o2's fft_lines_rd_from; two-stage sizes), 4 = mode 1
    with the fused order-2 rows' split (n = 48: LineFFT<48, INV, 8>).
    Returns the digit-reversal map (physical position -> logical index)."""
    assert data.dtype == np.complex64 and data.flags.c_contiguous
    perm = np.zeros(n, np.int32)
    check(load().wst_host_fft_lines(int(n), 1 if inverse else 0, int(mode), data.ctypes.data,
                                    int(nb), int(bs), int(nl), int(ls), int(es), int(threads),
                                    perm.ctypes.data))
    return perm


class Plan:
    """Owning handle of a ``wst_plan`` (bound to the device current at creation)."""

    def __init__(self, M, N, J, L, max_order=2, pre_pad=False, convention=None, lib=None):
        lib = lib or load()
        self._L = lib
        h = ctypes.c_void_p()
        self._chk(lib.wst_plan_create_ex(int(M), int(N), int(J), int(L), int(max_order),
                                     1 if pre_pad else 0, _conv_ptr(convention), ctypes.byref(h)))
        self._h = h
        K, Mo, No = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(lib.wst_output_shape(h, ctypes.byref(K), ctypes.byref(Mo), ctypes.byref(No)))
        self.K, self.Mo, self.No = K.value, Mo.value, No.value
        PM, PN = ctypes.c_int(), ctypes.c_int()
        self._chk(lib.wst_padded_shape(h, ctypes.byref(PM), ctypes.byref(PN)))
        self.PM, self.PN = PM.value, PN.value

    def _chk(self, code: int) -> None:
        """Status check against this plan's library (its thread-local last error)."""
        if code != WST_OK:
            raise WSTError(code, self._L.wst_last_error().decode(errors="replace") or f"wst status {code}")

    @property
    def handle(self):
        return self._h

    def workspace_bytes(self, nbatch: int) -> int:
        b = ctypes.c_size_t()
        self._chk(self._L.wst_workspace_bytes(self._h, int(nbatch), ctypes.byref(b)))
        return b.value

    def preferred_batch(self) -> int:
        """Planes per workspace chunk (wst_preferred_batch)."""
        b = ctypes.c_int64()
        self._chk(self._L.wst_preferred_batch(self._h, ctypes.byref(b)))
        return b.value

    def staging(self):
        """(rb, nst, sq) of the plan's level schedule (wst_plan_staging)."""
        rb, nst, sq = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self._L.wst_plan_staging(self._h, ctypes.byref(rb), ctypes.byref(nst), ctypes.byref(sq)))
        return rb.value, nst.value, sq.value

    def internal_workspaces(self):
        """(count, bytes) of the per-stream internal workspaces (wst_internal_workspaces)."""
        n, b = ctypes.c_int(), ctypes.c_size_t()
        self._chk(self._L.wst_internal_workspaces(self._h, ctypes.byref(n), ctypes.byref(b)))
        return n.value, b.value

    def forward(self, d_in: int, nbatch: int, d_out: int, pooled: bool, d_ws: int, ws_bytes: int,
                stream: int) -> None:
        self._chk(self._L.wst_forward(self._h, ctypes.c_void_p(d_in), int(nbatch),
                                 ctypes.c_void_p(d_out), 1 if pooled else 0,
                                 ctypes.c_void_p(d_ws or None), int(ws_bytes),
                                 ctypes.c_void_p(stream or None)))

    def forward_profiled(self, d_in: int, nbatch: int, d_out: int, pooled: bool, d_ws: int,
                         ws_bytes: int, stream: int, nslots: int):
        """wst_forward_profiled: returns per-kernel summed milliseconds (list of nslots)."""
        ms = (ctypes.c_float * nslots)()
        self._chk(self._L.wst_forward_profiled(self._h, ctypes.c_void_p(d_in), int(nbatch),
                                          ctypes.c_void_p(d_out), 1 if pooled else 0,
                                          ctypes.c_void_p(d_ws or None), int(ws_bytes),
                                          ctypes.c_void_p(stream or None), ms, nslots))
        return list(ms)

    def variants(self) -> np.ndarray:
        """Host-mirror trace words of one chunk (sites x 12, wst_plan_variants)."""
        n = ctypes.c_int64()
        self._chk(self._L.wst_plan_variants(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), np.int32)
        self._chk(self._L.wst_plan_variants(self._h, out.ctypes.data, out.size, ctypes.byref(n)))
        return out[:n.value].reshape(-1, 12)

    def trace(self, enable: bool) -> None:
        """Enable / disable the device variant trace (wst_plan_trace)."""
        self._chk(self._L.wst_plan_trace(self._h, 1 if enable else 0))

    def read_trace(self) -> np.ndarray:
        """Device trace words of the last traced forward (sites x 12, wst_plan_read_trace)."""
        n = ctypes.c_int64()
        self._chk(self._L.wst_plan_variants(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), np.int32)
        self._chk(self._L.wst_plan_read_trace(self._h, out.ctypes.data, out.size, ctypes.byref(n)))
        return out[:n.value].reshape(-1, 12)

    def close(self):
        if getattr(self, "_h", None) is not None and getattr(self, "_L", None) is not None:
            self._L.wst_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
