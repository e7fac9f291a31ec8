"""Generate the structured-pattern golden fixture at BASELINE config 5's geometry (256^2, one band,
J=6, L=12: P = 384, two HBM-staged levels, whose box-sparse folds keep 1-2 % of the alias taps) from
the float64 oracle, together with the fp32 noise floor of the reference algorithm on the same planes
(tests/patterns.py fp32_cascade: scipy single-precision pocketfft), so that the GPU test
(tests/test_gpu_patterns.py::test_structured_patterns_c5_geometry) needs neither the oracle nor the
fp32 cascade at test time.

Patterns (tests/patterns.py, after visualize_features.py:50-120): both gradients, the checkerboard,
the sharp-edged square and an impulse -- the inputs where the folds' dropped bins could bite.
Not listed in manifest.json (whose entries are the seeded uint8 goldens the parity tests enumerate);
the fixture carries its own geometry (J, L, the pattern names).
Run:  python tests/golden/make_pattern_golden.py       (~20 s on one core)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import kymatio_ref as kr  # noqa: E402
from parity import elementwise_error, per_coef_error  # noqa: E402
from patterns import fp32_cascade, patterns  # noqa: E402

NAME = "c5_patterns_256_J6_L12"
M, J, L = 256, 6, 12
PATTERNS = ["gradient_h", "gradient_v", "checkerboard", "edge", "impulse"]


def main():
    pats = patterns(M)
    x = np.stack([pats[k] for k in PATTERNS])           # (5, 256, 256) float32
    sc = kr.Scattering2D(J=J, shape=(M, M), L=L)
    S, f32_ew, f32_pc = [], [], []
    for i, name in enumerate(PATTERNS):
        t0 = time.time()
        ref = sc(x[i:i + 1])
        f32 = fp32_cascade(sc, x[i:i + 1])
        floor = 1e-3 if name.startswith("gradient") else 0.0
        S.append(ref[0])
        f32_ew.append(elementwise_error(f32, ref, floor=floor))
        f32_pc.append(per_coef_error(f32, ref, floor=floor))
        print(f"{name}: {time.time() - t0:.1f} s, fp32 pocketfft per-coefficient {f32_pc[-1].max():.2e}, "
              f"elementwise {f32_ew[-1].max():.2e}", flush=True)
    S = np.stack(S)
    np.savez_compressed(os.path.join(HERE, NAME + ".npz"), x=x, S=S.astype(np.float32),
                        names=np.array(PATTERNS), f32_elementwise=np.stack(f32_ew).astype(np.float32),
                        f32_per_coef=np.stack(f32_pc).astype(np.float32), J=J, L=L)


if __name__ == "__main__":
    main()
