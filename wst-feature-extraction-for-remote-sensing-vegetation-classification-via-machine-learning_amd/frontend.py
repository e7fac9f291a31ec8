"""Shared frontend logic: the kymatio 0.3.0 ``ScatteringBase2D`` contract + the GPU call.

Mirrors [kymatio 0.3.0] frontend/base_frontend.py (constructor signature, ``build`` checks,
padding) as used by the reference at src/training/train_and_save_model.py:359 and
src/inference/inference.py:242.  The arithmetic runs only in the HIP library (``_lib``).
"""
from __future__ import annotations

import threading

from . import _lib

_plan_cache: dict = {}
_plan_lock = threading.Lock()

# planes per workspace chunk: Xhat + the order-1 half spectra, 471 KB/plane at c2 (965 MB)
WORKSPACE_PLANES = 2048


def compute_padding(M: int, N: int, J: int) -> tuple[int, int]:
    """[kymatio 0.3.0] scattering2d/utils.py ``compute_padding``."""
    return ((M + 2 ** J) // 2 ** J + 1) * 2 ** J, ((N + 2 ** J) // 2 ** J + 1) * 2 ** J


def num_coefficients(J: int, L: int, max_order: int = 2) -> int:
    return 1 + J * L + (L * L * J * (J - 1) // 2 if max_order >= 2 else 0)


def _torch():
    import torch
    return torch


def require_gpu():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError(
            "wst_amd: no ROCm GPU is visible. The scattering transform runs only in the HIP "
            "extension (libwst_hip.so); there is no CPU fallback.")
    _lib.load()


def get_plan(device_index: int, M, N, J, L, max_order, pre_pad) -> _lib.Plan:
    key = (device_index, M, N, J, L, max_order, bool(pre_pad))
    plan = _plan_cache.get(key)
    if plan is not None:
        return plan
    with _plan_lock:
        plan = _plan_cache.get(key)
        if plan is None:
            torch = _torch()
            with torch.cuda.device(device_index):
                plan = _lib.Plan(M, N, J, L, max_order, pre_pad)
            _plan_cache[key] = plan
    return plan


def scatter_device(x, M, N, J, L, max_order, pre_pad, pooled=False, out=None):
    """Run the transform on a (B, h, w) float32 contiguous CUDA tensor.

    Returns (B, K, Mo, No) float32, or (B, 2K) [mean | std] when ``pooled``.
    Asynchronous on the current stream of ``x.device``."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 3
    dev = x.device.index if x.device.index is not None else torch.cuda.current_device()
    plan = get_plan(dev, M, N, J, L, max_order, pre_pad)
    B = x.shape[0]
    shape = (B, 2 * plan.K) if pooled else (B, plan.K, plan.Mo, plan.No)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=x.device)
    elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous():
        raise RuntimeError(f"out must be a contiguous float32 tensor of shape {shape}")
    if B == 0:
        return out
    planes = min(B, WORKSPACE_PLANES, plan.preferred_batch())
    ws_bytes = plan.workspace_bytes(planes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    # the plan is bound to x's device: make it current for the call (wst_forward checks it)
    with torch.cuda.device(dev):
        plan.forward(x.data_ptr(), B, out.data_ptr(), pooled, ws.data_ptr(), ws_bytes, stream)
    return out


class ScatteringBase2D:
    """[kymatio 0.3.0] ScatteringBase2D: same signature, same build-time checks."""

    def __init__(self, J, shape, L=8, max_order=2, pre_pad=False, backend=None,
                 out_type="array"):
        self.J, self.L, self.max_order = int(J), int(L), int(max_order)
        self.pre_pad, self.backend, self.out_type = pre_pad, backend, out_type
        self.shape = tuple(int(s) for s in shape)
        self.build()

    def build(self):
        if len(self.shape) != 2:
            raise RuntimeError("shape must be a 2-tuple (M, N).")
        M, N = self.shape
        self.M, self.N = M, N
        if 2 ** self.J > M or 2 ** self.J > N:
            raise RuntimeError("The smallest dimension should be larger than 2^J.")
        if self.J < 1:
            raise RuntimeError("J must be >= 1.")
        if self.max_order not in (1, 2):
            raise RuntimeError("max_order must be 1 or 2.")
        self._M_padded, self._N_padded = compute_padding(M, N, self.J)
        self.M_padded, self.N_padded = self._M_padded, self._N_padded
        self.K = num_coefficients(self.J, self.L, self.max_order)
        self.Mo, self.No = M // 2 ** self.J, N // 2 ** self.J

    # coefficient metadata in stack order (for out_type='list')
    def meta(self):
        items = [{"j": (), "theta": ()}]
        for j1 in range(self.J):
            for l1 in range(self.L):
                items.append({"j": (j1,), "theta": (l1,)})
        if self.max_order >= 2:
            for j1 in range(self.J):
                for l1 in range(self.L):
                    for j2 in range(j1 + 1, self.J):
                        for l2 in range(self.L):
                            items.append({"j": (j1, j2), "theta": (l1, l2)})
        return items

    def _check_spatial(self, shape, kind):
        if len(shape) < 2:
            raise RuntimeError(f"Input {kind} must have at least two dimensions.")
        if (shape[-1] != self.N or shape[-2] != self.M) and not self.pre_pad:
            raise RuntimeError(f"{kind} must be of spatial size ({self.M},{self.N}).")
        if (shape[-1] != self._N_padded or shape[-2] != self._M_padded) and self.pre_pad:
            raise RuntimeError(f"Padded {kind} must be of spatial size "
                               f"({self._M_padded},{self._N_padded}).")
        if self.out_type not in ("array", "list"):
            raise RuntimeError("The out_type must be one of 'array' or 'list'.")

    def _to_list(self, S, batch_shape):
        out = []
        for k, m in enumerate(self.meta()):
            out.append({"coef": S[..., k, :, :], "j": m["j"], "theta": m["theta"]})
        return out
