"""NumPy frontend: drop-in for ``from kymatio.numpy import Scattering2D``.

Reference call sites: src/training/train_and_save_model.py:46,359,368 and
src/visualization/visualize_features.py:30.  The array is staged to the GPU (H2D), transformed
by the HIP library, and copied back (D2H).

Dtypes (kymatio.numpy's contract): the result is float64 for every real input.  kymatio's numpy
backend multiplies the input's spectrum by float64 filters, so a float32 input -- what the
reference passes, train_and_save_model.py:51-56,368 -- comes back float64, and its np.mean /
np.std at :371-372 then accumulate in float64.  The transform itself computes in float32 on the
GPU (a float64 input is rounded to float32 on the way in); the returned values carry float32
precision, within the per-coefficient 1e-5 tolerance of the float64 reference (tests/parity.py).
"""
from __future__ import annotations

import numpy as np

from .frontend import ScatteringBase2D, require_gpu, scatter_device


class Scattering2D(ScatteringBase2D):
    """Scattering2D(J, shape, L=8, max_order=2, pre_pad=False, backend=None, out_type='array')."""

    def scattering(self, input):
        if not isinstance(input, np.ndarray):
            raise TypeError("The input should be a NumPy array.")
        if np.iscomplexobj(input):
            raise TypeError("The input should be real.")
        self._check_spatial(input.shape, "array")
        require_gpu()
        import torch
        batch_shape = input.shape[:-2]
        x = np.ascontiguousarray(input, dtype=np.float32).reshape((-1,) + input.shape[-2:])
        xd = torch.from_numpy(x).to("cuda", non_blocking=False)
        S = scatter_device(xd, self.M, self.N, self.J, self.L, self.max_order, self.pre_pad)
        S = S.cpu().numpy().astype(np.float64)   # kymatio.numpy returns float64 (see above)
        S = S.reshape(batch_shape + S.shape[-3:])
        if self.out_type == "list":
            return self._to_list(S, batch_shape)
        return S

    def pooled(self, input):
        """Per-coefficient spatial [mean | std] (population std): (..., 2K) float64, the dtype of
        the reference's np.mean / np.std over kymatio.numpy's output (computed in float32)."""
        if not isinstance(input, np.ndarray):
            raise TypeError("The input should be a NumPy array.")
        self._check_spatial(input.shape, "array")
        require_gpu()
        import torch
        batch_shape = input.shape[:-2]
        x = np.ascontiguousarray(input, dtype=np.float32).reshape((-1,) + input.shape[-2:])
        xd = torch.from_numpy(x).to("cuda")
        F = scatter_device(xd, self.M, self.N, self.J, self.L, self.max_order, self.pre_pad,
                           pooled=True)
        F = F.cpu().numpy().reshape(batch_shape + (2 * self.K,))
        return F.astype(np.float64)

    __call__ = scattering
