"""Error profile of the structured patterns (dev tool): per pattern, the largest |S_gpu - S_ref|
relative to the plane's strongest coefficient, and the per-coefficient error with the
denominator floored at F x (strongest coefficient) for several F."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np
from oracle import kymatio_ref as kr
from test_gpu_patterns import patterns
from parity import elementwise_error
from wst_amd.numpy import Scattering2D as NpS
for n, J in [(128, 2), (64, 4)]:
    pats = patterns(n)
    x = np.stack(list(pats.values()))
    got = NpS(J=J, shape=(n, n), L=8)(x).astype(np.float64)
    ref = kr.Scattering2D(J=J, shape=(n, n), L=8)(x)
    for i, name in enumerate(pats):
        g, r = got[i].reshape(got.shape[1], -1), ref[i].reshape(ref.shape[1], -1)
        top = np.abs(r).max()
        dk = np.abs(g - r).max(axis=1)
        sk = np.abs(r).max(axis=1)
        line = f"{n} J={J} {name:16s} abs/top {dk.max() / top:.2e}"
        for F in (0, 1e-6, 1e-5, 1e-4, 1e-3):
            sc = np.maximum(sk, F * top)
            sc = np.where(sc > 0, sc, 1.0)
            line += f"  F={F:g}: {(dk / sc).max():.2e}"
        for sig in (1e-3, 1e-2):
            ew = elementwise_error(got[i:i + 1], ref[i:i + 1], significant=sig, floor=1e-3)
            line += f"  ew@{sig:g}: {ew.max():.2e}"
        print(line, flush=True)
