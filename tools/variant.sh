#!/bin/bash
# Build a library variant that differs only in one family pair's kernels (A/B dev tool):
#   [PAIR=17_17] tools/variant.sh <name> <extra hipcc flags...>   ->  <pkg>/var_<name>.so  (AB_LIB=var_<name>.so)
# (-DWST_DIAG variants also need the host side: VARIANT_HOST=1 recompiles wst_hip.hip with the flags;
#  HOST_ONLY=1: only wst_hip.hip with the flags, production kernels -- e.g. the env A/B knobs of -DWST_DIAG)
name=$1; shift
pair=${PAIR:-3_3}; fm=${pair%_*}; fn=${pair#*_}
pkg=wst-feature-extraction-for-remote-sensing-vegetation-classification-via-machine-learning_amd
cd "$(dirname "$0")/../$pkg/csrc" || exit 1
mkdir -p ../../build_var   # objects; the .so goes next to libwst_hip.so
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result"
if [ -n "$HOST_ONLY" ]; then
  VARIANT_HOST=1
  objs=$(ls ../build/*.o)
else
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize -DWST_FAM_M=$fm -DWST_FAM_N=$fn "$@" -c -o ../../build_var/kern_${pair}_$name.o wst_kernels.hip || exit 1
  objs="$(ls ../build/*.o | grep -v "kern_${pair}.o") ../../build_var/kern_${pair}_$name.o"
fi
if [ -n "$VARIANT_HOST" ]; then
  /opt/rocm/bin/hipcc $F "$@" -c -o ../../build_var/wst_hip_$name.o wst_hip.hip || exit 1
  objs="$(echo $objs | tr ' ' '\n' | grep -v wst_hip.o) ../../build_var/wst_hip_$name.o"
fi
/opt/rocm/bin/hipcc $F -shared -o ../var_$name.so $objs
echo built $pkg/var_$name.so "(AB_LIB=var_$name.so)"
