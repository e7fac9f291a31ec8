#!/bin/bash
# Alternating A/B of library variants (GPU box; dev tool): tools/ab_rep.sh <tag> <planes,M,J> <reps> lib1.so lib2.so ...
tag=$1; geom=$2; reps=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
for r in $(seq 1 $reps); do
  for l in "$@"; do
    dump=""; [ $r = 1 ] && dump=gpurun_out/${tag}_out_${l%.so}.npy
    KM_DUMP=$dump WST_KM_GEOM=$geom AB_LIB=$l timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/${tag}_km_${l}_$r.txt 2>&1 || { echo "$l failed"; tail -5 gpurun_out/${tag}_km_${l}_$r.txt; exit 99; }
    echo "$r $(tail -1 gpurun_out/${tag}_km_${l}_$r.txt)"
  done
done
# every library's outputs against the first one's (same input planes): max per-coefficient
# relative difference, a cross-check that an A/B arm computes the same transform
python3 - "$tag" "$@" <<'PY' || exit 99
import sys, numpy as np
tag, libs = sys.argv[1], sys.argv[2:]
ref = np.load(f"gpurun_out/{tag}_out_{libs[0][:-3]}.npy").astype(np.float64)
r = ref.reshape(ref.shape[0], ref.shape[1], -1)
for l in libs[1:]:
    o = np.load(f"gpurun_out/{tag}_out_{l[:-3]}.npy").astype(np.float64).reshape(r.shape)
    d = (np.abs(o - r).max(axis=(0, 2)) / np.maximum(np.abs(r).max(axis=(0, 2)), 1e-30)).max()
    print(f"[ab_rep] {l} vs {libs[0]}: max per-coefficient rel diff {d:.3e}")
    if not d < 1e-5: sys.exit(f"{l} differs from {libs[0]}")
PY
