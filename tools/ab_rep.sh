#!/bin/bash
# Alternating A/B of library variants (GPU box; dev tool): tools/ab_rep.sh <tag> <planes,M,J> <reps> lib1.so lib2.so ...
tag=$1; geom=$2; reps=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
for r in $(seq 1 $reps); do
  for l in "$@"; do
    WST_KM_GEOM=$geom AB_LIB=$l timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/${tag}_km_${l}_$r.txt 2>&1 || { echo "$l failed"; tail -5 gpurun_out/${tag}_km_${l}_$r.txt; exit 99; }
    echo "$r $(tail -1 gpurun_out/${tag}_km_${l}_$r.txt)"
  done
done
