"""Every reachable kernel variant against the float64 oracle, and the device's own account of
which variant it ran (tests/test_variants_cpu.py proves the cover reaches them all).

For each geometry of tests/variant_geometries.py: one uint8/255 plane (regenerated from its seed)
  * through the trace build (libwst_hip_trace.so: the same sources with -DWST_TRACE; the product
    library carries no trace code) with the device trace on (wst_plan_trace): the words the
    kernels wrote == the host mirror's prediction (wst_plan_variants);
  * through the product library: the coefficients at the fixture's sampled positions (all of them for maps <= 16 values)
    meet the parity bar against the oracle's (tests/golden/variants_cover.npz,
    make_variant_golden.py): per coefficient max |d| / max |S_ref[k]| <= TOL, and elementwise on
    the significant entries (|S_ref| >= 1e-3 max |S_ref[k]|).
"""
import os

import numpy as np
import pytest
import torch

from parity import SIGNIFICANT, TOL
from variant_geometries import COVER

import wst_amd  # noqa: F401
from wst_amd import _lib, variants

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = np.load(os.path.join(HERE, "golden", "variants_cover.npz"))


def _plane(g):
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_variant_golden as mvg
    return mvg.plane_of(g)


@pytest.mark.parametrize("i", range(len(COVER)), ids=[f"{g[0]}x{g[1]}_J{g[2]}_L{g[3]}_o{g[4]}" for g in COVER])
def test_variant_geometry_matches_oracle_and_mirror(i):
    g = tuple(int(v) for v in FIX["geoms"][i])
    assert g == tuple(COVER[i])
    M, N, J, L, mo = g
    x = torch.from_numpy(_plane(g)).cuda()

    def run(plan):
        out = torch.empty((1, plan.K, plan.Mo, plan.No), device="cuda")
        ws = torch.empty(plan.workspace_bytes(1), dtype=torch.uint8, device="cuda")
        plan.forward(x.data_ptr(), 1, out.data_ptr(), False, ws.data_ptr(), ws.numel(),
                     torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return out

    plan = _lib.Plan(M, N, J, L, mo, False)                          # the product library
    out = run(plan)
    tplan = _lib.Plan(M, N, J, L, mo, False, lib=_lib.load_trace())   # the trace build
    tplan.trace(True)
    tout = run(tplan)
    dev, mirror = tplan.read_trace(), plan.variants()
    assert np.array_equal(tplan.variants(), mirror)
    # the trace build computes what the product computes (its trace stores are the only difference)
    assert torch.equal(out, tout), f"{g}: trace build and product differ"
    if not np.array_equal(dev, mirror):
        bad = [s for s in range(len(mirror)) if not np.array_equal(dev[s], mirror[s])]
        raise AssertionError(f"{g}: device ran another variant than the mirror predicts at sites {bad[:4]}: "
                             f"device {variants.describe(dev[bad[:1]])} mirror {variants.describe(mirror[bad[:1]])}")
    got = out[0].reshape(plan.K, -1).cpu().numpy().astype(np.float64)[:, FIX[f"{i}_pos"]]
    ref = FIX[f"{i}_ref"].astype(np.float64)
    scale = FIX[f"{i}_scale"].astype(np.float64)
    assert got.shape == ref.shape
    den = np.where(scale > 0, scale, 1.0)
    err = np.abs(got - ref).max(axis=1) / den
    k = int(np.argmax(err))
    assert err.max() <= TOL, f"{g}: per-coefficient rel err {err.max():.3e} at k={k} ({variants.describe(mirror)})"
    sig = np.abs(ref) >= SIGNIFICANT * scale[:, None]
    ew = np.where(sig & (ref != 0), np.abs(got - ref) / np.where(ref != 0, np.abs(ref), 1.0), 0.0)
    assert ew.max() <= TOL, f"{g}: elementwise rel err {ew.max():.3e} on significant entries"
    tplan.trace(False)


def test_product_library_has_no_trace_code():
    """wst_plan_trace is refused by the product library: its kernels carry no trace stores."""
    plan = _lib.Plan(64, 64, 4, 8)
    with pytest.raises(_lib.WSTError):
        plan.trace(True)
