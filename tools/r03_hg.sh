#!/bin/bash
# c5 HG k_o2 mapping A/B: WST_HG_SPLIT x WST_HG_GROUP (diag library), ms/step + HG kernel stats
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
lib=var_diag.so
for cfgs in "3 1" "10 1" "10 8" "10 32" "5 16" "10 64"; do
  set -- $cfgs
  WST_LIB=$lib WST_HG_SPLIT=$1 WST_HG_GROUP=$2 timeout -k 10 200 python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/$tag/b_$1_$2.log 2>&1 || exit 9
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$tag/b_$1_$2.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('split $1 group $2', d['ms_per_step'], {a: round(b,3) for a,b in k.items()})"
done
for cfgs in "3 1" "10 32"; do
  set -- $cfgs
  WST_LIB=$lib WST_HG_SPLIT=$1 WST_HG_GROUP=$2 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$tag/f_$1_$2 -o pmc -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 > gpurun_out/$tag/f_$1_$2.log 2>&1 || exit 9
done
echo done
