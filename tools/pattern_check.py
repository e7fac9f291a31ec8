"""Errors of one library build on the c5-geometry structured-pattern golden (dev tool, GPU box):
per plane the per-coefficient and elementwise errors against the fixture and the fixture's fp32
pocketfft errors (tests/golden/make_pattern_golden.py).  A/B of builds that differ in an
approximation (e.g. the box threshold): AB_LIB=<lib> python3 tools/pattern_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import wst_amd  # noqa: E402,F401
from wst_amd import _lib  # noqa: E402
if os.environ.get("AB_LIB"):
    _lib.use_library(os.environ["AB_LIB"])
from wst_amd.numpy import Scattering2D  # noqa: E402
from parity import elementwise_error, per_coef_error  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "c5_patterns_256_J6_L12.npz"))
got = Scattering2D(J=int(d["J"]), shape=d["x"].shape[-2:], L=int(d["L"]))(d["x"])
ref = d["S"].astype(np.float64)
for i, n in enumerate(str(v) for v in d["names"]):
    floor = 1e-3 if n.startswith("gradient") else 0.0
    g, r = got[i:i + 1], ref[i:i + 1]
    print(f"{os.environ.get('AB_LIB', 'libwst_hip.so')} {n}: per-coefficient {per_coef_error(g, r, floor).max():.3e} "
          f"(fp32 pocketfft {d['f32_per_coef'][i].max():.3e}), elementwise {elementwise_error(g, r, floor=floor).max():.3e} "
          f"(fp32 pocketfft {d['f32_elementwise'][i].max():.3e})", flush=True)
