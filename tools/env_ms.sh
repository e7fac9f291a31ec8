#!/bin/bash
# Per-kernel timings of one geometry under diagnostic-library env settings (dev tool, GPU box).
# usage: tools/env_ms.sh planes,M,J "VAR=value ..." ...   ("-" = no setting)
cd "$GRAFT_REPO_ROOT" || exit 99
g=$1; shift
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e WST_LIB=libwst_hip_diag.so WST_KM_GEOM=$g timeout -k 10 120 python3 tools/kernel_ms.py 2>&1 | tail -1 | sed "s/^/[$e] /" || exit 99
done
