#!/bin/bash
# A/B per-kernel HIP-event ms of library variants at one geometry (GPU box; dev tool):
#   tools/ab_km.sh <tag> <planes,M,J> lib1.so lib2.so ...   -> gpurun_out/<tag>_km_<lib>.txt
tag=$1; geom=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
for l in "$@"; do
  WST_KM_GEOM=$geom AB_LIB=$l timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/${tag}_km_$l.txt 2>&1 || { echo "$l failed"; tail -5 gpurun_out/${tag}_km_$l.txt; exit 99; }
  echo "$geom $(tail -1 gpurun_out/${tag}_km_$l.txt)"
done
