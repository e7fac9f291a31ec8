#!/bin/bash
# Build a library variant that differs only in the family-3 kernels (A/B dev tool):
#   tools/variant.sh <name> <extra hipcc flags...>   ->  build_var/<name>.so  (run with WST_LIB=...)
name=$1; shift
pkg=wst-feature-extraction-for-remote-sensing-vegetation-classification-via-machine-learning_amd
cd "$(dirname "$0")/../$pkg/csrc" || exit 1
mkdir -p ../../build_var # objects; the .so goes next to libwst_hip.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result \
  -fno-slp-vectorize -DWST_FAM_M=3 -DWST_FAM_N=3 "$@" -c -o ../../build_var/kern_3_3_$name.o wst_kernels.hip || exit 1
objs=$(ls ../build/*.o | grep -v kern_3_3.o)
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ../var_$name.so $objs ../../build_var/kern_3_3_$name.o
echo built $pkg/var_$name.so "(WST_LIB=var_$name.so)"
