#!/bin/bash
# k_o2 / k_o1 workgroup-size A/B on the c2 geometry with the diagnostic library (dev tool, GPU box).
# usage: tools/thr_ab.sh "O2=512" "O2=640" "O1=768,256" ...   (WST_O2_THREADS / WST_O1_THREADS lists)
cd "$GRAFT_REPO_ROOT" || exit 99
for v in "$@"; do
  o1=""; o2=""
  case $v in O1=*) o1=${v#O1=};; O2=*) o2=${v#O2=};; esac
  WST_LIB=libwst_hip_diag.so WST_O1_THREADS=$o1 WST_O2_THREADS=$o2 timeout -k 10 120 python3 tools/kernel_ms.py 2>&1 | tail -1 | sed "s/^/$v /" || exit 99
done
