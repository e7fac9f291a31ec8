#!/bin/bash
# f3 export-mode k_o2: batch split x group A/B (diag library) + FETCH of the best candidates
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
for r in 1 2; do
for cfgs in "1 1" "2 1" "4 1" "2 8" "4 8" "4 16" "2 32"; do
  set -- $cfgs
  WST_LIB=var_diag17.so WST_O2X_SPLIT=$1 WST_O2X_GROUP=$2 WST_KM_GEOM=768,128,2 timeout -k 10 120 python3 tools/kernel_ms.py 768 2>&1 | grep chunk | sed "s/^/split $1 group $2 /" || exit 9
done
done
for cfgs in "1 1" "4 8" "2 8"; do
  set -- $cfgs
  WST_LIB=var_diag17.so WST_O2X_SPLIT=$1 WST_O2X_GROUP=$2 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$tag/f_$1_$2 -o pmc -- python3 bench.py --config f3 --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 > gpurun_out/$tag/f_$1_$2.log 2>&1 || exit 9
done
echo done
