#!/bin/bash
# c5 staged / HG knob sweep on the diagnostic build (kernel_ms per-kernel HIP-event ms per step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
run() { name=$1; shift
  env "$@" AB_LIB=libwst_hip_diag.so WST_KM_GEOM=256,256,6,12 timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/r05q_$name.txt 2>&1 || { echo "$name failed"; tail -3 gpurun_out/r05q_$name.txt; exit 99; }
  echo "$name $(tail -1 gpurun_out/r05q_$name.txt)"; }
run base WST_DUMMY=0
run fa1 WST_FOLD_ALL=1
run fa4 WST_FOLD_ALL=4
run sp2 WST_HG_SPLIT=2
run sp8 WST_HG_SPLIT=8
run gr8 WST_HG_GROUP=8
run gr32 WST_HG_GROUP=32
run base2 WST_DUMMY=0
