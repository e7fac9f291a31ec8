"""Decoding of the kernel-variant trace words (include/wst_hip.h wst_plan_variants /
wst_describe_variants / wst_plan_read_trace; encoding: csrc/wst_device.h tr_*).

A forward launches a fixed sequence of kernels per chunk ("sites"); every site names the kernel
instantiation it runs, the body that instantiation dispatches to at run time and, for k_o2, the
branch each order-2 level takes.  `variant_keys` turns a (sites x 12) word array into the set of
code paths a geometry exercises; tests/test_variants_cpu.py proves the GPU oracle tests' geometries
reach every key any geometry can reach, tests/test_gpu_variants.py that the device runs exactly
what the host mirror predicts.
"""
from __future__ import annotations

import numpy as np

KINDS = {1: "k_prep", 2: "k_o1", 3: "k_o2", 4: "k_big_rows", 5: "k_big_cols"}
LP = {0: "taps", 1: "mfma_rc", 2: "mfma", 3: "plain"}
FOLD2 = {1: "fused_s2_rowA", 2: "tile_s2", 3: "tile_list", 4: "dense_s2", 5: "box"}
FOLD1 = {0: "fused_rowA", 1: "s1", 2: "s2", 3: "box", 4: "s4", 5: "runtime_s"}
SPEC = {0: "hbm", 1: "rd_from", 2: "copy"}
BRANCH = {1: "N1C", 2: "hg_ct_export", 3: "hg_ct_first", 4: "hg_runtime", 5: "exp_ct", 6: "exp_runtime",
          7: "runtime"}
ROWMODE = {0: "pad", 1: "real2", 2: "fold1", 3: "fold2", 4: "half"}
COLMODE = {0: "store", 1: "modlp", 2: "modlp_fwd"}


def _bits(v, lo, n):
    return (int(v) >> lo) & ((1 << n) - 1)


def kernel_name(w0):
    kind = _bits(w0, 28, 3)
    fm, fn, cap, sq, hg = _bits(w0, 22, 6), _bits(w0, 16, 6), _bits(w0, 4, 12), _bits(w0, 1, 1), _bits(w0, 0, 1)
    name = KINDS.get(kind, f"kind{kind}")
    if kind == 1:
        return f"{name}<{fm}, {fn}>"
    if kind == 2:
        return f"{name}<{fm}, {fn}, {cap}, {sq}>"
    if kind == 3:
        return f"{name}<{fm}, {fn}, {cap}, {sq}, {hg}>"
    return f"{name}<{cap}, {'true' if hg else 'false'}>"


def body_name(w0, w1):
    kind = _bits(w0, 28, 3)
    if kind == 1:
        return f"PC={_bits(w1, 0, 8)} lp={LP[_bits(w1, 8, 2)]}"
    if kind == 2:
        return (f"OC={_bits(w1, 0, 4)} N1C={_bits(w1, 4, 8)} fused1={_bits(w1, 12, 1)} "
                f"lp={LP[_bits(w1, 13, 2)]} do2={_bits(w1, 15, 1)} export={_bits(w1, 16, 1)} "
                f"fold={FOLD1.get(_bits(w1, 17, 3), '?')}")
    if kind == 3:
        return (f"OC={_bits(w1, 0, 4)} LC={_bits(w1, 4, 5)} N1C={_bits(w1, 9, 8)} "
                f"spec={SPEC.get(_bits(w1, 17, 2), '?')} branch={BRANCH.get(_bits(w1, 19, 3), '?')}")
    mode = _bits(w1, 0, 3)
    if kind == 4:
        return (f"mode={ROWMODE.get(mode, mode)} fold_all={_bits(w1, 3, 1)} fold1={_bits(w1, 4, 2)} "
                f"box={_bits(w1, 6, 1)}")
    return f"mode={COLMODE.get(mode, mode)} wide={_bits(w1, 7, 1)} g_lds={_bits(w1, 8, 1)} u={_bits(w1, 9, 1)}"


def level_name(wl):
    """The code path of an order-2 level.  The alias count s is not part of it: the dense form is
    s = 2 by construction, the box form takes s at run time (one code path for every s >= 4)."""
    fold = _bits(wl, 7, 3)
    sc = _bits(wl, 18, 3)
    s = f"PB={_bits(wl, 21, 5)} SC={(1 << sc) if sc else 0} NC={_bits(wl, 10, 8)} fold={FOLD2.get(fold, '?')} " \
        f"lp={LP[_bits(wl, 5, 2)]}"
    return s


def site_keys(row):
    """Variant keys of one site: the kernel + body, and one per order-2 level it runs."""
    w0, w1 = int(row[0]), int(row[1])
    if w0 == 0:
        return set()
    base = f"{kernel_name(w0)} [{body_name(w0, w1)}]"
    keys = {base}
    for wl in row[2:]:
        if int(wl) & 1:
            keys.add(f"{base} level[{level_name(int(wl))}]")
    return keys


def variant_keys(words) -> set:
    keys = set()
    for row in np.asarray(words).reshape(-1, 12):
        keys |= site_keys(row)
    return keys


def describe(words) -> list:
    """Readable lines, one per site (and its levels)."""
    out = []
    for row in np.asarray(words).reshape(-1, 12):
        if int(row[0]) == 0:
            out.append("(untraced)")
            continue
        line = f"{kernel_name(row[0])} [{body_name(row[0], row[1])}]"
        lv = [f"j2={_bits(w, 26, 5)} s={1 << _bits(w, 1, 4)}: {level_name(int(w))}" for w in row[2:] if int(w) & 1]
        out.append(line + ("  " + "; ".join(lv) if lv else ""))
    return out
