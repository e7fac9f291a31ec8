#!/bin/bash
# Per-kernel timings of the c2 / c1 / f3 geometries for the given libraries (dev tool, GPU box).
# usage: tools/geo_ms.sh lib.so [lib2.so ...]
cd "$GRAFT_REPO_ROOT" || exit 99
for lib in "$@"; do
  for g in "3072,64,4 c2" "3072,64,2 c1" "768,128,2 f3"; do
    set -- $g
    WST_LIB=$lib WST_KM_GEOM=$1 timeout -k 10 120 python3 tools/kernel_ms.py 2>&1 | tail -1 | sed "s/^/$2 /" || exit 99
  done
done
