#!/bin/bash
# c5 HG split sweep on the diagnostic build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
run() { name=$1; shift
  env "$@" AB_LIB=libwst_hip_diag.so WST_KM_GEOM=256,256,6,12 timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/r05r_$name.txt 2>&1 || { echo "$name failed"; tail -3 gpurun_out/r05r_$name.txt; exit 99; }
  echo "$name $(tail -1 gpurun_out/r05r_$name.txt)"; }
run sp4 WST_HG_SPLIT=4
run sp2 WST_HG_SPLIT=2
run sp1 WST_HG_SPLIT=1
run sp3 WST_HG_SPLIT=3
run sp21 WST_HG_SPLIT=2,1
run sp12 WST_HG_SPLIT=1,2
run sp2g8 WST_HG_SPLIT=2 WST_HG_GROUP=8
run sp2g32 WST_HG_SPLIT=2 WST_HG_GROUP=32
run sp2b WST_HG_SPLIT=2
