"""CPU restatement of the reference's operators either side of the WST path -- TEST
INFRASTRUCTURE ONLY (same rule as oracle/kymatio_ref.py: only tests/, smoke() and bench.py's
cpu_baseline may import it; the product path never does).

* Noise injection, ``src/preprocessing/add_noise.py:14-72``.  Every
  function takes the random draws explicitly, so the formula part is deterministic and can be
  checked bit-for-bit against the GPU kernels fed the same draws; ``draw_*`` reproduce the
  reference's own draws with numpy's legacy global RNG (np.random.normal / randn / poisson /
  uniform / randint, exactly as add_noise.py calls them).
* advanced_stats (row F4), ``src/training/train_and_save_model.py:58-112``: restated with the
  same numpy / scipy calls (scipy.stats.skew / kurtosis, scipy.ndimage.sobel / laplace) on the
  same float32 channels; ``extract_hybrid_features`` follows :380-387.

Pinning: these are line-by-line restatements of reference code whose only dependencies
(numpy 2.2, scipy 1.15) are importable here; the golden fixtures under tests/golden/ are
generated from them by tests/golden/make_aux_golden.py.
"""
from __future__ import annotations

import numpy as np
from scipy import stats
from scipy.ndimage import laplace, sobel

NOISE_TYPES = ("gaussian", "salt_and_pepper", "speckle", "poisson", "uniform")


# --------------------------------------------------------------------------------------------
# noise formulas (draws supplied) -- add_noise.py:14-72
# --------------------------------------------------------------------------------------------
def gaussian_formula(image_array, gauss):
    """add_noise.py:14-21: clip(image + gauss, 0, 255).astype(uint8), gauss ~ N(0, I*255/100)."""
    noisy = image_array + gauss
    return np.clip(noisy, 0, 255).astype(np.uint8)


def salt_and_pepper_formula(image_array, salt_rc, pepper_rc):
    """add_noise.py:23-42: salt rows/cols -> 255 in every channel, then pepper -> 0."""
    noisy = np.copy(image_array)
    noisy[salt_rc[0], salt_rc[1], :] = 255
    noisy[pepper_rc[0], pepper_rc[1], :] = 0
    return noisy


def speckle_formula(image_array, gauss, intensity):
    """add_noise.py:44-53: clip(image + image * randn * I/100)."""
    noise_factor = intensity / 100
    noisy = image_array + image_array * gauss * noise_factor
    return np.clip(noisy, 0, 255).astype(np.uint8)


def poisson_scale(intensity):
    return 10 + (intensity / 100) * 90


def poisson_formula(image_array, draws, intensity):
    """add_noise.py:55-63: clip(poisson(image * sf / 255) * 255 / sf), sf = 10 + 0.9 I."""
    scale_factor = poisson_scale(intensity)
    noisy = draws * 255.0 / scale_factor
    return np.clip(noisy, 0, 255).astype(np.uint8)


def uniform_formula(image_array, noise):
    """add_noise.py:65-71: clip(image + U(-r/2, r/2)), r = I*255/100."""
    noisy = image_array + noise
    return np.clip(noisy, 0, 255).astype(np.uint8)


def salt_and_pepper_counts(shape, intensity):
    size = int(np.prod(shape))
    amount = intensity / 100
    return int(np.ceil(amount * size * 0.5)), int(np.ceil(amount * size * (1. - 0.5)))


# --------------------------------------------------------------------------------------------
# the reference's own draws (numpy legacy global RNG, same calls and order as add_noise.py)
# --------------------------------------------------------------------------------------------
def draw(noise_type, image_array, intensity):
    """Returns the draws add_noise.py would make for `image_array` (HWC uint8)."""
    row, col, ch = image_array.shape
    if noise_type == "gaussian":
        return np.random.normal(0, intensity * 255 / 100, (row, col, ch))
    if noise_type == "speckle":
        return np.random.randn(row, col, ch).reshape(row, col, ch)
    if noise_type == "poisson":
        scaled = image_array * poisson_scale(intensity) / 255.0
        return np.random.poisson(scaled).astype(np.float64)
    if noise_type == "uniform":
        r = intensity * 255 / 100
        return np.random.uniform(-r / 2, r / 2, (row, col, ch))
    if noise_type == "salt_and_pepper":
        ns, npp = salt_and_pepper_counts(image_array.shape, intensity)
        salt = [np.random.randint(0, i - 1, ns) for i in image_array.shape]
        pepper = [np.random.randint(0, i - 1, npp) for i in image_array.shape]
        return (np.stack(salt[:2]).astype(np.int32), np.stack(pepper[:2]).astype(np.int32))
    raise ValueError(f"Unknown noise type: {noise_type}")


def apply(noise_type, image_array, intensity, draws):
    if noise_type == "gaussian":
        return gaussian_formula(image_array, draws)
    if noise_type == "speckle":
        return speckle_formula(image_array, draws, intensity)
    if noise_type == "poisson":
        return poisson_formula(image_array, draws, intensity)
    if noise_type == "uniform":
        return uniform_formula(image_array, draws)
    if noise_type == "salt_and_pepper":
        return salt_and_pepper_formula(image_array, draws[0], draws[1])
    raise ValueError(f"Unknown noise type: {noise_type}")


# --------------------------------------------------------------------------------------------
# advanced_stats -- train_and_save_model.py:58-112 (per channel, 18 features)
# --------------------------------------------------------------------------------------------
STAT_NAMES = ('mean', 'std', 'var', 'min', 'max', 'range', 'skew', 'kurt', 'cv',
              'p10', 'p25', 'p50', 'p75', 'p90', 'iqr', 'mad', 'grad_mean', 'edge_density')


def extract_advanced_features(rgb_image):
    """(C, H, W) float32 -> (C*18,) float64, exactly the reference's calls."""
    C = rgb_image.shape[0]
    fpc = 18
    features = np.zeros(C * fpc)
    for i in range(C):
        channel = rgb_image[i]
        ch_flat = channel.ravel()
        ch_clean = ch_flat[np.isfinite(ch_flat)]
        if len(ch_clean) == 0:
            continue
        base = i * fpc
        features[base + 0] = np.mean(ch_clean)
        features[base + 1] = np.std(ch_clean)
        features[base + 2] = np.var(ch_clean)
        features[base + 3] = np.min(ch_clean)
        features[base + 4] = np.max(ch_clean)
        features[base + 5] = np.ptp(ch_clean)
        features[base + 6] = stats.skew(ch_clean)
        features[base + 7] = stats.kurtosis(ch_clean)
        mean_val = features[base + 0]
        features[base + 8] = features[base + 1] / max(mean_val, 1e-8)
        features[base + 9] = np.percentile(ch_clean, 10)
        features[base + 10] = np.percentile(ch_clean, 25)
        features[base + 11] = np.percentile(ch_clean, 50)
        features[base + 12] = np.percentile(ch_clean, 75)
        features[base + 13] = np.percentile(ch_clean, 90)
        features[base + 14] = features[base + 12] - features[base + 10]
        features[base + 15] = np.mean(np.abs(ch_clean - mean_val))
        try:
            grad_x = sobel(channel, axis=0)
            grad_y = sobel(channel, axis=1)
            grad_mag = np.sqrt(grad_x ** 2 + grad_y ** 2)
            features[base + 16] = np.mean(grad_mag.ravel())
            edges = np.abs(laplace(channel))
            edge_thr = np.percentile(edges.ravel(), 90)
            features[base + 17] = np.mean(edges.ravel() > edge_thr)
        except Exception:
            features[base + 16] = 0
            features[base + 17] = 0
    return features


def extract_hybrid_features(rgb_image, wst_features):
    """train_and_save_model.py:380-387: [advanced (C*18) | wst (C*2K)]."""
    return np.concatenate([extract_advanced_features(rgb_image), wst_features])


MOMENT_IDX = (0, 1, 2, 6, 7, 8, 15)   # mean, std, var, skew, kurt, cv, mad


def advanced_moments_f64(rgb_image):
    """The moment features of extract_advanced_features computed exactly (float64 data): the
    reference evaluates them in float32 (numpy / scipy keep the input dtype), which is off from
    the exact values by up to ~4e-4 relative for skew; the GPU computes them in float64.
    Returns (C, 7) in MOMENT_IDX order."""
    out = []
    for ch in rgb_image:
        c = ch.ravel().astype(np.float64)
        c = c[np.isfinite(c)]
        m = c.mean()
        sd = c.std()
        out.append([m, sd, c.var(), stats.skew(c), stats.kurtosis(c), sd / max(m, 1e-8),
                    np.mean(np.abs(c - m))])
    return np.array(out)
