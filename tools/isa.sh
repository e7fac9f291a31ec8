#!/bin/bash
# Device assembly of one family pair's kernels (dev tool): tools/isa.sh [PAIR=3_3] [extra flags] -> /tmp/isa/kern_<pair>.s
pair=${PAIR:-3_3}; fm=${pair%_*}; fn=${pair#*_}
cd "$(dirname "$0")/../wst-feature-extraction-for-remote-sensing-vegetation-classification-via-machine-learning_amd/csrc" || exit 1
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -fno-slp-vectorize \
  -DWST_FAM_M=$fm -DWST_FAM_N=$fn "$@" --cuda-device-only -S -o /tmp/isa/kern_$pair.s wst_kernels.hip
