"""Error bound of the box-sparse folds' threshold (test infrastructure, CPU; csrc/wst_hip.hip
kBoxThreshold): zero every psi Fourier bin below thr x its filter level's maximum in the float64
oracle and report the largest change of the output -- an upper bound for the folds, whose alias
boxes keep every bin inside a window around the significant ones (a superset of the bins above thr).

Two input families:
* random uint8 planes (the goldens' inputs) at c2 (64^2 J=4), f3 (128^2 J=2) and c5 (256^2 J=6 L=12);
* the structured patterns of tests/patterns.py (visualize_features.py:50-120: gradients,
  checkerboard, sharp-edged square, impulse) at c5's geometry, where the s = 16 / 32 folds keep only
  1-2 % of the alias taps.  Reported with the parity metrics of tests/parity.py: per-coefficient
  change (gradients: denominator floored at 1e-3 of the strongest coefficient) and elementwise change
  on the significant entries.
usage: python tests/golden/box_threshold.py [random] [patterns]      (c5 patterns: ~2 min per threshold)
"""
import copy
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import kymatio_ref as kr  # noqa: E402
from parity import elementwise_error, per_coef_error  # noqa: E402
from patterns import patterns  # noqa: E402


def masked(S, thr):
    S2 = copy.deepcopy(S)
    kept = []
    for psi in S2.psi:
        for r, f in enumerate(psi["levels"]):
            mask = np.abs(f) > thr * np.abs(f).max()
            kept.append(mask.mean())
            psi["levels"][r] = np.where(mask, f, 0.0)
    return S2, float(np.mean(kept))


def run_random(M, J, L, thrs, nplanes=2, seed=0):
    S = kr.Scattering2D(J, (M, M), L)
    x = np.random.default_rng(seed).integers(0, 256, (nplanes, M, M)).astype(np.float64) / 255
    ref = S.scattering(x)
    for thr in thrs:
        S2, kept = masked(S, thr)
        out = S2.scattering(x)
        print(f"random M={M} J={J} L={L} thr={thr:.0e}: per-coefficient change {per_coef_error(out, ref).max():.2e}, "
              f"elementwise {elementwise_error(out, ref).max():.2e} (mean kept bins {kept:.3f})", flush=True)


def run_patterns(M, J, L, thrs, names=("gradient_h", "gradient_v", "checkerboard", "edge", "impulse")):
    S = kr.Scattering2D(J, (M, M), L)
    pats = patterns(M)
    x = np.stack([pats[n] for n in names]).astype(np.float64)
    ref = S.scattering(x)
    for thr in thrs:
        S2, kept = masked(S, thr)
        out = S2.scattering(x)
        for i, n in enumerate(names):
            floor = 1e-3 if n.startswith("gradient") else 0.0
            o, r = out[i:i + 1], ref[i:i + 1]
            print(f"{n} M={M} J={J} L={L} thr={thr:.0e}: per-coefficient change "
                  f"{per_coef_error(o, r, floor).max():.2e}, elementwise {elementwise_error(o, r, floor=floor).max():.2e} "
                  f"(mean kept bins {kept:.3f})", flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["random", "patterns"]
    if "random" in what:
        run_random(64, 4, 8, [1e-10, 1e-9, 1e-8, 1e-7, 1e-6])
        run_random(128, 2, 8, [1e-10, 1e-8, 1e-7, 1e-6])
        run_random(256, 6, 12, [1e-10, 1e-8, 1e-7], nplanes=1)
    if "patterns" in what:
        run_patterns(256, 6, 12, [1e-10, 1e-8, 1e-7])
