#!/bin/bash
# c5 workgroup-size sweep of the HG k_o2 (staged j1 = 0, 1) and the resident k_o2 at j1 = 2 (diagnostic build)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
run() { name=$1; shift
  env "$@" AB_LIB=libwst_hip_diag.so WST_KM_GEOM=256,256,6,12 timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/r05z_$name.txt 2>&1 || { echo "$name failed"; tail -3 gpurun_out/r05z_$name.txt; exit 99; }
  echo "$name $(tail -1 gpurun_out/r05z_$name.txt)"; }
run base WST_DUMMY=0
run hg512 WST_HG_THREADS=512,512
run hg768 WST_HG_THREADS=768,768
run hg1024 WST_HG_THREADS=1024,1024
run o2_768 WST_O2_THREADS=64,64,768
run o2_1024 WST_O2_THREADS=64,64,1024
run base2 WST_DUMMY=0
