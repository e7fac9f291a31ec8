#!/bin/bash
# Phase ablation of one geometry with the diagnostic library (dev tool, GPU box): WST_DEBUG_SKIP
# masks skip kernel phases (results invalid, timings only).  usage: tools/skip_ab.sh planes,M,J mask...
cd "$GRAFT_REPO_ROOT" || exit 99
g=$1; shift
for m in "$@"; do
  WST_LIB=libwst_hip_diag.so WST_KM_GEOM=$g WST_DEBUG_SKIP=$m timeout -k 10 120 python3 tools/kernel_ms.py 2>&1 | tail -1 | sed "s/^/skip=$m /" || exit 99
done
