"""Error bound of the box-sparse folds' threshold (dev tool, CPU): zero every psi Fourier bin below
thr x the filter level's maximum in the float64 oracle and report the largest per-coefficient change
(relative to the coefficient's maximum over the planes) -- an upper bound for the folds, whose alias
boxes keep every bin inside a window around the significant ones.  csrc/wst_hip.hip kBoxThreshold."""
import sys, numpy as np, copy, time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import kymatio_ref as kr
def run(M, J, L, thrs, nplanes=2, seed=0):
    S = kr.Scattering2D(J, (M, M), L)
    x = np.random.default_rng(seed).integers(0, 256, (nplanes, M, M)).astype(np.float64) / 255
    ref = S.scattering(x)
    scale = np.abs(ref).reshape(nplanes, ref.shape[1], -1).max(axis=(0, 2))
    for thr in thrs:
        S2 = copy.deepcopy(S)
        kept = []
        for psi in S2.psi:
            for r, f in enumerate(psi["levels"]):
                m = np.abs(f).max()
                mask = np.abs(f) > thr * m
                kept.append(mask.mean())
                psi["levels"][r] = np.where(mask, f, 0.0)
        out = S2.scattering(x)
        err = (np.abs(out - ref).reshape(nplanes, ref.shape[1], -1).max(axis=(0, 2)) / np.where(scale > 0, scale, 1)).max()
        print(f"M={M} J={J} L={L} thr={thr:.0e}: max per-coefficient rel err {err:.2e} (mean kept bins {np.mean(kept):.3f})", flush=True)
run(64, 4, 8, [1e-10, 1e-9, 1e-8, 1e-7, 1e-6])
run(128, 2, 8, [1e-10, 1e-8, 1e-7, 1e-6])
run(256, 6, 12, [1e-10, 1e-8, 1e-7], nplanes=1)
