"""Every kernel variant a geometry can select is oracle-tested (CPU side; no GPU).

The library's host mirror of the kernels' run-time dispatch (wst_describe_variants, a plan built
without a GPU) names, per launch, the kernel instantiation, the body it dispatches to and the
branch of every order-2 level (wst_amd.variants).  tools/variant_cover.py walked a sweep of
33k geometries in padded-size space (every square P to 584 and a grid to 1204, J 1..8,
L in {1, 2, 3, 7, 8, 12}, orders 1 and 2; rectangular pairs with J 1..5, L in {3, 8}) and
stored the reachable set in tests/golden/variant_universe.json; tests/variant_geometries.py is
a cover of it, which tests/test_gpu_variants.py runs on the GPU against the float64 oracle and
checks the device trace against the mirror.  Here:
  * the cover reaches every reachable variant;
  * a fresh sweep reaches nothing outside the stored set (a code change that adds a variant
    fails here until the cover is regenerated);
  * the library compiles exactly the reachable k_o1 / k_o2 / k_prep / staged instantiations
    (csrc/wst_compiled.h, generated from the same sweep);
  * a seeded random sweep OFF that grid (L in 4..16 outside the grid's values, rectangular planes
    with J up to 8) selects only compiled kernels: no plan fails with "not compiled", and every
    kernel it names is in the library (guards a dispatch change that only affects off-grid L / J).
"""
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import wst_amd  # noqa: F401
from wst_amd import _lib, variants
from variant_geometries import COVER

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
UNIVERSE = json.load(open(os.path.join(HERE, "golden", "variant_universe.json")))


def _sweep():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import variant_cover
    return variant_cover.sweep_geometries()


def test_describe_runs_without_gpu_and_names_the_headline_kernels():
    lines = variants.describe(_lib.describe_variants(64, 64, 4, 8))     # BASELINE config 2
    assert lines[0] == "k_prep<3, 3> [PC=96 lp=plain]"
    assert lines[2].startswith("k_o2<3, 3, 136, 1, 0> [OC=4 LC=8 N1C=96 spec=rd_from branch=N1C]")
    assert "j2=1 s=2: PB=2 SC=2 NC=48 fold=fused_s2_rowA lp=taps" in lines[2]
    f3 = variants.describe(_lib.describe_variants(128, 128, 2, 8))      # the reference's geometry
    assert f3[2].startswith("k_o2<17, 17, 136, 0, 1> [OC=0 LC=8 N1C=0 spec=hbm branch=exp_ct]")
    c5 = variants.describe(_lib.describe_variants(256, 256, 6, 12))     # BASELINE config 5
    assert c5[0].startswith("k_big_rows<384, false> [mode=pad")
    assert sum("k_big_rows<192, true> [mode=fold2 fold_all=1" in s for s in c5) == 12


def test_cover_reaches_every_reachable_variant():
    universe = set(UNIVERSE["keys"])
    covered = set()
    for g in COVER:
        covered |= variants.variant_keys(_lib.describe_variants(*g))
    missing = sorted(universe - covered)
    assert not missing, f"{len(missing)} reachable variants no GPU oracle test reaches, e.g. {missing[:3]}"


@pytest.mark.parametrize("cfg", [(64, 64, 2, 8), (64, 64, 4, 8), (256, 256, 6, 12), (128, 128, 2, 8)])
def test_baseline_configs_are_in_the_cover(cfg):
    covered = set()
    for g in COVER:
        covered |= variants.variant_keys(_lib.describe_variants(*g))
    assert variants.variant_keys(_lib.describe_variants(*cfg)) <= covered


def test_sweep_reaches_nothing_outside_the_stored_universe():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import variant_cover
    universe = set(UNIVERSE["keys"])
    seen, _ = variant_cover.reachable(_sweep())       # host-only plans in a fork pool (no GPU)
    new = sorted(seen - universe)
    assert not new, (f"{len(new)} variants outside tests/golden/variant_universe.json (rerun "
                     f"tools/variant_cover.py --write and tests/golden/make_variant_golden.py): {new[:3]}")
    assert seen == universe


def _compiled_kernels():
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-C", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    names = set()
    for m in re.finditer(r"(?:wstdev|wstbig)::(k_(?:prep|o1|o2|big_rows|big_cols)<[^>]*>)\(", out):
        names.add(m.group(1))
    return names


def test_compiled_kernels_are_exactly_the_reachable_ones():
    """wst_compiled.h (tools/variant_cover.py) lists the k_o1 / k_o2 instantiations some geometry
    selects; the library carries those and no other (a plan selecting another fails at creation)."""
    compiled = _compiled_kernels()
    reached = {k.split(" [")[0] for k in UNIVERSE["keys"]}
    assert compiled == reached, (sorted(compiled - reached)[:5], sorted(reached - compiled)[:5])


def _offgrid_geometries(n=1500, seed=6):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        J = int(rng.integers(1, 9))
        s = 1 << J
        L = int(rng.choice([4, 5, 6, 9, 10, 11, 13, 14, 15, 16]))
        mo = int(rng.integers(1, 3))
        hi = 1204 // s
        PM = s * int(rng.integers(3, hi + 1))
        PN = PM if rng.random() < 0.4 else s * int(rng.integers(3, hi + 1))
        out.append((PM - 2 * s, PN - 2 * s, J, L, mo))
    return out


def _describe_or_error(g):
    try:
        return g, sorted(variants.variant_keys(_lib.describe_variants(*g))), None
    except _lib.WSTError as e:
        return g, None, str(e)


def test_offgrid_geometries_select_only_compiled_kernels():
    import multiprocessing as mp
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(_describe_or_error, _offgrid_geometries(), chunksize=32)
    uncompiled = [(g, e) for g, _, e in res if e and "not compiled" in e]
    assert not uncompiled, f"{len(uncompiled)} off-grid geometries hit an uncompiled kernel, e.g. {uncompiled[:2]}"
    compiled = _compiled_kernels()
    named = {k.split(" [")[0] for _, keys, _ in res if keys for k in keys}
    assert named <= compiled, sorted(named - compiled)[:5]
    valid = sum(keys is not None for _, keys, _ in res)
    assert valid > 500, valid     # the sweep mostly reaches plannable geometries
