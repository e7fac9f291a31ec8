"""Device-side data paths either side of the transform.

* ``generate_patches`` -- synthetic uint8/255 patches keyed by (seed, global patch index)
  (``wst_patch_generate``): the c3 workload generates 1M patches on the GPUs, each rank its
  own contiguous shard, and a patch's values never depend on the world size or the chunking.
* ``u8_hwc_to_chw`` -- batched ``load_rgb_image`` conversion (train_and_save_model.py:51-56,
  inference.py:163-168): uint8 (B, H, W, C) PIL arrays -> float32 (B, C, H, W) / 255 on the
  device (``wst_u8_to_chw``), the input layout of the WST path.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .frontend import require_gpu

OUT_KINDS = {"uint8": 0, "float": 1}


def generate_patches(seed: int, first: int, n: int, C: int, H: int, W: int, device=None,
                     out: str = "float", dst=None):
    """Patches [first, first + n) as a (n, C, H, W) device tensor: float32 values k/255
    (``out='float'``) or the uint8 bytes k (``out='uint8'``).  ``dst`` (optional) receives them."""
    import torch
    require_gpu()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    dt = torch.float32 if out == "float" else torch.uint8
    if dst is None:
        dst = torch.empty((n, C, H, W), dtype=dt, device=dev)
    elif dst.dtype != dt or not dst.is_contiguous() or dst.numel() < n * C * H * W:
        raise RuntimeError(f"dst must be a contiguous {dt} tensor of >= {n * C * H * W} elements")
    with torch.cuda.device(dst.device):
        _lib.check_aux(_lib.load().wst_patch_generate(int(seed) & (2 ** 64 - 1), int(first), int(n),
                                                      int(C), int(H), int(W), OUT_KINDS[out],
                                                      dst.data_ptr(),
                                                      torch.cuda.current_stream(dst.device).cuda_stream))
    return dst


def u8_hwc_to_chw(images, device=None):
    """(B, H, W, C) uint8 (numpy or torch) -> float32 (B, C, H, W) / 255 on the GPU."""
    import torch
    require_gpu()
    if isinstance(images, np.ndarray):
        if images.dtype != np.uint8:
            raise TypeError("images must be uint8")
        t = torch.from_numpy(np.ascontiguousarray(images)).to(device or "cuda")
    else:
        if images.dtype != torch.uint8:
            raise TypeError("images must be uint8")
        t = images.contiguous()
        if not t.is_cuda:
            t = t.to(device or "cuda")
    if t.dim() == 3:
        t = t[..., None]
    if t.dim() != 4:
        raise RuntimeError("images must be (B, H, W, C)")
    B, H, W, C = t.shape
    out = torch.empty((B, C, H, W), dtype=torch.float32, device=t.device)
    with torch.cuda.device(t.device):
        _lib.check_aux(_lib.load().wst_u8_to_chw(t.data_ptr(), B, H, W, C, out.data_ptr(),
                                                 torch.cuda.current_stream(t.device).cuda_stream))
    return out
