"""Torch frontend: drop-in for ``from kymatio.torch import Scattering2D``.

Reference call site: src/inference/inference.py:39,242,250-254 (``S(channel_tensor)`` on a
contiguous float32 ``(1,1,H,W)`` tensor under ``torch.no_grad()``).  CUDA (ROCm) tensors are
transformed in place on their device with zero copies; CPU tensors are staged to the current
GPU and the result is returned on the CPU, so the reference's CPU-tensor call keeps working.
Gradients are not implemented (the reference only runs the transform under no_grad).
"""
from __future__ import annotations

import torch

from .frontend import ScatteringBase2D, require_gpu, scatter_device


class Scattering2D(ScatteringBase2D, torch.nn.Module):
    """Scattering2D(J, shape, L=8, max_order=2, pre_pad=False, backend=None, out_type='array')."""

    def __init__(self, J, shape, L=8, max_order=2, pre_pad=False, backend=None,
                 out_type="array"):
        torch.nn.Module.__init__(self)
        ScatteringBase2D.__init__(self, J, shape, L, max_order, pre_pad, backend, out_type)

    def _prepare(self, input):
        if not torch.is_tensor(input):
            raise TypeError("The input should be a PyTorch Tensor.")
        if input.is_complex():
            raise TypeError("The input should be real.")
        self._check_spatial(tuple(input.shape), "tensor")
        if not input.is_contiguous():
            raise RuntimeError("Tensor must be contiguous.")
        require_gpu()
        batch_shape = tuple(input.shape[:-2])
        x = input.detach().reshape((-1,) + tuple(input.shape[-2:]))
        if x.dtype != torch.float32:
            x = x.to(torch.float32)
        on_cpu = not x.is_cuda
        if on_cpu:
            x = x.to("cuda")
        return x.contiguous(), batch_shape, on_cpu

    def scattering(self, input):
        x, batch_shape, on_cpu = self._prepare(input)
        with torch.no_grad():
            S = scatter_device(x, self.M, self.N, self.J, self.L, self.max_order, self.pre_pad)
        if on_cpu:
            S = S.cpu()
        S = S.reshape(batch_shape + tuple(S.shape[-3:]))
        if self.out_type == "list":
            return self._to_list(S, batch_shape)
        return S

    def pooled(self, input):
        """Per-coefficient spatial [mean | std] (population std): (..., 2K) float32."""
        x, batch_shape, on_cpu = self._prepare(input)
        with torch.no_grad():
            F = scatter_device(x, self.M, self.N, self.J, self.L, self.max_order, self.pre_pad,
                               pooled=True)
        if on_cpu:
            F = F.cpu()
        return F.reshape(batch_shape + (2 * self.K,))

    def forward(self, input):
        return self.scattering(input)

    def __call__(self, input):
        return self.scattering(input)
