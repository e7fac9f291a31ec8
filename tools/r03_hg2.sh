#!/bin/bash
# c5 HG k_o2 split x group A/B, two passes each, + FETCH of the candidates (diag library)
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
lib=var_diag.so
for pass in 1 2; do
for cfgs in "3 1" "5 16" "5 8" "4 16" "5 32" "6 8"; do
  set -- $cfgs
  WST_LIB=$lib WST_HG_SPLIT=$1 WST_HG_GROUP=$2 timeout -k 10 200 python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/$tag/b.log 2>&1 || exit 9
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$tag/b.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('pass $pass split $1 group $2', d['ms_per_step'], 'o2 j1=0', k['k_o2_j1=0'], 'j1=1', k['k_o2_j1=1'])"
done
done
for cfgs in "5 16" "4 16" "6 8"; do
  set -- $cfgs
  WST_LIB=$lib WST_HG_SPLIT=$1 WST_HG_GROUP=$2 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$tag/f_$1_$2 -o pmc -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 > gpurun_out/$tag/f_$1_$2.log 2>&1 || exit 9
done
echo done
