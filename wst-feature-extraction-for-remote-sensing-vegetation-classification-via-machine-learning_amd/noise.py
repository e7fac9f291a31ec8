"""Noise injection of the reference's robustness sweep on the GPU.

Mirrors ``src/preprocessing/add_noise.py:14-72``: the same five noise types, intensity
conventions and uint8 clipping.  The function names of the reference
(``add_gaussian_noise(image_array, intensity)`` ...) take and return HWC uint8 numpy arrays;
``add_noise_batch`` is the batched device form used by the c4 sweep, which can emit the WST input
directly (float32 CHW / 255, the ``load_rgb_image`` convention of train_and_save_model.py:51-56).

Randomness: the production path draws on the device (Philox4x32-10 keyed by seed, image and
element) -- numpy's global MT19937 stream is not reproduced.  ``apply_noise_draws`` runs the
identical kernel formulas on caller-supplied draws, which is how the parity tests show the GPU
formulas are bit-exact with the reference's.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .frontend import require_gpu

NOISE_TYPES = {"gaussian": 0, "salt_and_pepper": 1, "speckle": 2, "poisson": 3, "uniform": 4}
OUT_KINDS = {"uint8_hwc": 0, "float_chw": 1}


def _type_id(noise_type):
    try:
        return NOISE_TYPES[noise_type]
    except KeyError:
        raise ValueError(f"Unknown noise type: {noise_type}") from None   # add_noise.py:94


def _device_u8(images):
    import torch
    require_gpu()
    if isinstance(images, np.ndarray):
        if images.dtype != np.uint8:
            raise TypeError("images must be uint8 (PIL HWC arrays)")
        t = torch.from_numpy(np.ascontiguousarray(images)).to("cuda")
    else:
        if images.dtype != torch.uint8:
            raise TypeError("images must be uint8 (PIL HWC arrays)")
        t = images.to("cuda") if not images.is_cuda else images
        t = t.contiguous()
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if t.dim() != 4:
        raise RuntimeError("images must be (H, W, C) or (B, H, W, C)")
    return t


def _out(t, out):
    import torch
    B, H, W, C = t.shape
    if OUT_KINDS[out] == 0:
        return torch.empty((B, H, W, C), dtype=torch.uint8, device=t.device)
    return torch.empty((B, C, H, W), dtype=torch.float32, device=t.device)


def salt_pepper_counts(H, W, C, intensity):
    ns, npp = ctypes.c_int64(), ctypes.c_int64()
    _lib.check_aux(_lib.load().wst_salt_pepper_counts(int(H), int(W), int(C), float(intensity),
                                                      ctypes.byref(ns), ctypes.byref(npp)))
    return ns.value, npp.value


def add_noise_batch(images, noise_type, intensity, seed=0, out="uint8_hwc"):
    """(B, H, W, C) uint8 -> noisy batch on the device: uint8 HWC (``out='uint8_hwc'``) or the
    float32 CHW / 255 WST input (``out='float_chw'``)."""
    import torch
    t = _device_u8(images)
    B, H, W, C = t.shape
    o = _out(t, out)
    st = torch.cuda.current_stream(t.device).cuda_stream
    with torch.cuda.device(t.device):
        _lib.check_aux(_lib.load().wst_noise_generate(_type_id(noise_type), float(intensity),
                                                      t.data_ptr(), B, H, W, C,
                                                      int(seed) & (2 ** 64 - 1), OUT_KINDS[out],
                                                      o.data_ptr(), st))
    return o


def apply_noise_draws(images, noise_type, intensity, draws, out="uint8_hwc"):
    """The kernel formulas on given draws: ``draws`` is the float64 noise array add_noise.py
    draws (gaussian / speckle / poisson / uniform, shape (B, H, W, C)) or, for salt and pepper,
    a pair of int32 (B, 2, count) row/column arrays (salt, pepper)."""
    import torch
    t = _device_u8(images)
    B, H, W, C = t.shape
    o = _out(t, out)
    st = torch.cuda.current_stream(t.device).cuda_stream
    tid = _type_id(noise_type)
    if tid == NOISE_TYPES["salt_and_pepper"]:
        salt, pepper = (torch.as_tensor(np.ascontiguousarray(a, np.int32)).reshape(B, 2, -1)
                        .to(t.device) for a in draws)
        ns, npp = salt_pepper_counts(H, W, C, intensity)
        if salt.shape[-1] != ns or pepper.shape[-1] != npp:
            raise RuntimeError(f"salt/pepper counts must be {ns}/{npp}")
        with torch.cuda.device(t.device):
            code = _lib.load().wst_noise_apply(tid, float(intensity), t.data_ptr(), B, H, W, C,
                                               None, salt.data_ptr(), pepper.data_ptr(),
                                               OUT_KINDS[out], o.data_ptr(), st)
    else:
        d = torch.as_tensor(np.ascontiguousarray(draws, np.float64)).reshape(B, H, W, C).to(t.device)
        with torch.cuda.device(t.device):
            code = _lib.load().wst_noise_apply(tid, float(intensity), t.data_ptr(), B, H, W, C,
                                               d.data_ptr(), None, None, OUT_KINDS[out],
                                               o.data_ptr(), st)
    _lib.check_aux(code)
    return o


def _single(noise_type, image_array, intensity, seed):
    if seed is None:
        seed = int(np.random.randint(0, 2 ** 31 - 1))
    return add_noise_batch(np.asarray(image_array)[None], noise_type, intensity, seed)[0].cpu().numpy()


# drop-in names of add_noise.py (HWC uint8 in, HWC uint8 out)
def add_gaussian_noise(image_array, intensity, seed=None):
    """add_noise.py:14-21."""
    return _single("gaussian", image_array, intensity, seed)


def add_salt_and_pepper_noise(image_array, intensity, seed=None):
    """add_noise.py:23-42."""
    return _single("salt_and_pepper", image_array, intensity, seed)


def add_speckle_noise(image_array, intensity, seed=None):
    """add_noise.py:44-53."""
    return _single("speckle", image_array, intensity, seed)


def add_poisson_noise(image_array, intensity, seed=None):
    """add_noise.py:55-63."""
    return _single("poisson", image_array, intensity, seed)


def add_uniform_noise(image_array, intensity, seed=None):
    """add_noise.py:65-71."""
    return _single("uniform", image_array, intensity, seed)
