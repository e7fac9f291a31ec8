"""Structured input planes (the synthetic patterns of the reference's visualisation,
src/visualization/visualize_features.py:50-120 -- gradients, checkerboard, concentric circles, random
and striped textures, a sharp-edged square -- plus an impulse) and the fp32 noise floor of the
reference algorithm on them.  Test infrastructure: used by tests/test_gpu_patterns.py,
tests/golden/make_pattern_golden.py and tools/box_threshold.py.

The generators are this repository's own restatement of those pattern definitions (input data
only).  They exercise what random uint8 noise does not: constant rows / columns meeting the reflect
padding (gradients), energy concentrated at the highest frequencies (checkerboard), a single bin
(impulse) and large flat regions with sharp edges.
"""
import numpy as np


def patterns(n):
    t = np.linspace(0.0, 1.0, n)
    out = {
        "gradient_h": np.tile(t, (n, 1)),
        "gradient_v": np.tile(t[:, None], (1, n)),
    }
    sq = n // 8
    ij = np.add.outer(np.arange(n) // sq, np.arange(n) // sq)
    out["checkerboard"] = (ij % 2 == 0).astype(np.float64)
    yy, xx = np.mgrid[0:n, 0:n]
    r = np.hypot(yy - n / 2, xx - n / 2) / (n / 2)
    out["circles"] = np.sin(r * 5 * np.pi) * 0.5 + 0.5
    rng = np.random.RandomState(42)
    out["texture"] = rng.rand(n, n)
    stripes = (np.sin(np.linspace(0, 8 * 2 * np.pi, n))[None, :].repeat(n, 0) + 1) / 2
    out["vertical_texture"] = np.clip(stripes * 0.7 + rng.rand(n, n) * 0.3, 0, 1)
    edge = np.zeros((n, n))
    b = n * 20 // 128
    edge[b:n - b, b:n - b] = 1.0
    out["edge"] = edge
    imp = np.zeros((n, n))
    imp[n // 3, n // 2] = 1.0
    out["impulse"] = imp
    return {k: v.astype(np.float32) for k, v in out.items()}


def fp32_cascade(sc, x):
    """The oracle's cascade (kymatio_ref.scattering2d) run with float32 input and filters, so every
    FFT is scipy's single-precision pocketfft: the fp32 noise floor of the reference algorithm."""
    from oracle import kymatio_ref as kr

    def f32(d):
        return {**d, "levels": [np.asarray(v, np.float32) for v in d["levels"]]}
    out = kr.scattering2d(np.asarray(x, np.float32), lambda v: kr.reflect_pad(v, sc.pad_size),
                          sc.J, sc.L, f32(sc.phi), [f32(p) for p in sc.psi], sc.max_order)
    assert out.dtype == np.float32
    return out
