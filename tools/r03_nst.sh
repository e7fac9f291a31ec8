#!/bin/bash
# c5: staged/HG split point A/B (WST_NST) + parity of the variant
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
lib=var_diag.so
for cfgs in "2 3 1" "3 3 1" "3 5 16" "2 5 16"; do
  set -- $cfgs
  WST_LIB=$lib WST_NST=$1 WST_HG_SPLIT=$2 WST_HG_GROUP=$3 timeout -k 10 200 python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/$tag/b_$1_$2_$3.log 2>&1 || exit 9
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$tag/b_$1_$2_$3.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('nst $1 split $2 group $3', d['ms_per_step'], d.get('parity'), {a: round(b,3) for a,b in k.items() if 'o2' in a or 'o1_j1=0' in a})"
done
WST_LIB=$lib WST_NST=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_staged.py -m gpu -q -x -k "c5 or staged_batch" --timeout 200 --timeout-method thread > gpurun_out/$tag/pytest.txt 2>&1; tail -2 gpurun_out/$tag/pytest.txt
