"""WST feature layouts of the reference's callers (row F1 of SURVEY.md §8(f)).

* Training layout -- src/training/train_and_save_model.py:346-378: per channel
  ``[mean_k (K) | std_k (K)]`` (population std over the (Mo, No) map), channels concatenated:
  C * 2K features (486 for RGB at J=2, L=8).  Names follow get_feature_names :400-427, with
  the hard-coded 81 replaced by the true K for any (J, L).
* Inference layout -- src/inference/inference.py:237-270: per channel interleaved
  ``[m_0, s_0, m_1, s_1, ...]``.

The pooling is fused into the HIP kernels' epilogue (pooled=1): only 2K floats per plane leave
the GPU instead of K*Mo*No.

Row F4: ``advanced_stats`` (train_and_save_model.py:58-112, 18 features per channel, one
workgroup per plane in csrc/wst_aux.hip) and ``hybrid`` = [advanced | wst] (:380-387);
``extract_features`` / ``get_feature_names`` accept the reference's method strings (:389-427).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .frontend import require_gpu, scatter_device, num_coefficients

CHANNEL_NAMES = ("R", "G", "B")
STAT_NAMES = ('mean', 'std', 'var', 'min', 'max', 'range', 'skew', 'kurt', 'cv',
              'p10', 'p25', 'p50', 'p75', 'p90', 'iqr', 'mad', 'grad_mean', 'edge_density')


def get_feature_names(J=2, L: int = 8, channels=CHANNEL_NAMES, max_order: int = 2):
    """``{ch}_wst_{mean|std}_{k}`` in training order (channel -> stat -> k).

    Called with a method string, as the reference does (``get_feature_names('hybrid')``,
    train_and_save_model.py:400-427): 'advanced_stats' -> ``{ch}_{stat}``; 'wst' -> the WST
    names for (J=2, L=8) with the true K (81) instead of the hard-coded 81; 'hybrid' -> both."""
    if isinstance(J, str):
        method = J
        if method == "advanced_stats":
            return [f"{c}_{s}" for c in channels for s in STAT_NAMES]
        if method == "wst":
            return get_feature_names(2, 8, channels, max_order)
        if method == "hybrid":
            return get_feature_names("advanced_stats", channels=channels) + \
                get_feature_names(2, 8, channels, max_order)
        raise ValueError(f"Unknown feature method: {method}")
    K = num_coefficients(J, L, max_order)
    return [f"{c}_wst_{s}_{i}" for c in channels for s in ("mean", "std") for i in range(K)]


def _pooled_batch(images, J, L, max_order):
    """images: (B, C, H, W) numpy or torch -> torch (B, C, 2K) float32 on the GPU."""
    import torch
    require_gpu()
    if isinstance(images, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(images, dtype=np.float32)).to("cuda")
    else:
        x = images.detach().to(device="cuda" if not images.is_cuda else images.device,
                                dtype=torch.float32).contiguous()
    if x.dim() != 4:
        raise RuntimeError("images must be (B, C, H, W)")
    B, C, H, W = x.shape
    F = scatter_device(x.reshape(B * C, H, W), H, W, J, L, max_order, False, pooled=True)
    return F.reshape(B, C, -1)


def extract_wst_features_batch(images, J: int = 2, L: int = 8, max_order: int = 2,
                               as_numpy: bool = True):
    """Training-layout features for a batch: (B, C, H, W) -> (B, C*2K).

    One GPU call replaces the reference's B*C serial kymatio calls
    (train_and_save_model.py:486-488 x :364-376)."""
    F = _pooled_batch(images, J, L, max_order)
    F = F.reshape(F.shape[0], -1)
    return F.cpu().numpy().astype(np.float64) if as_numpy else F


def extract_wst_features(rgb_image, J: int = 2, L: int = 8):
    """Drop-in for train_and_save_model.py:346-378 ``extract_wst_features(rgb_image)``:
    (C, H, W) float -> (C*2K,) float64."""
    return extract_wst_features_batch(np.asarray(rgb_image)[None], J, L)[0]


def extract_wst_features_interleaved_batch(images, J: int = 2, L: int = 8, max_order: int = 2,
                                           as_numpy: bool = True):
    """Inference layout (inference.py:263-266): per channel [m_0, s_0, m_1, s_1, ...]."""
    F = _pooled_batch(images, J, L, max_order)          # (B, C, 2K) = [means | stds]
    B, C, K2 = F.shape
    K = K2 // 2
    inter = F.reshape(B, C, 2, K).transpose(2, 3).reshape(B, C * 2 * K)
    return inter.cpu().numpy().astype(np.float64) if as_numpy else inter


def extract_wst_features_interleaved(rgb_image, J: int = 2, L: int = 8):
    """Drop-in for inference.py:237-270 ``ModelInference.extract_wst_features``."""
    return extract_wst_features_interleaved_batch(np.asarray(rgb_image)[None], J, L)[0]


def _device_planes(images):
    import torch
    require_gpu()
    if isinstance(images, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(images, dtype=np.float32)).to("cuda")
    else:
        x = images.detach().to(device="cuda" if not images.is_cuda else images.device,
                                dtype=torch.float32).contiguous()
    if x.dim() != 4:
        raise RuntimeError("images must be (B, C, H, W)")
    return x


def extract_advanced_features_batch(images, as_numpy: bool = True):
    """advanced_stats for a batch: (B, C, H, W) float32 -> (B, C*18) float64, per channel the
    18 statistics of train_and_save_model.py:58-112 (one GPU workgroup per plane)."""
    import torch
    x = _device_planes(images)
    B, C, H, W = x.shape
    out = torch.empty((B * C, 18), dtype=torch.float64, device=x.device)
    with torch.cuda.device(x.device):
        _lib.check_aux(_lib.load().wst_advanced_stats(x.data_ptr(), B * C, H, W, out.data_ptr(),
                                                      torch.cuda.current_stream(x.device).cuda_stream))
    out = out.reshape(B, C * 18)
    return out.cpu().numpy() if as_numpy else out


def extract_advanced_features(rgb_image):
    """Drop-in for train_and_save_model.py:58-112 ``extract_advanced_features(rgb_image)``."""
    return extract_advanced_features_batch(np.asarray(rgb_image)[None])[0]


def extract_hybrid_features_batch(images, J: int = 2, L: int = 8):
    """hybrid = [advanced_stats (C*18) | wst (C*2K)] per image (train_and_save_model.py:380-387)."""
    x = _device_planes(images)
    return np.concatenate([extract_advanced_features_batch(x), extract_wst_features_batch(x, J, L)], 1)


def extract_hybrid_features(rgb_image, J: int = 2, L: int = 8):
    """Drop-in for train_and_save_model.py:380-387 ``extract_hybrid_features(rgb_image)``."""
    return extract_hybrid_features_batch(np.asarray(rgb_image)[None], J, L)[0]


def extract_features(rgb_image, feature_method):
    """Drop-in for train_and_save_model.py:389-398 ``extract_features(rgb_image, method)``."""
    if feature_method == "advanced_stats":
        return extract_advanced_features(rgb_image)
    if feature_method == "wst":
        return extract_wst_features(rgb_image)
    if feature_method == "hybrid":
        return extract_hybrid_features(rgb_image)
    raise ValueError(f"Unknown feature method: {feature_method}")
