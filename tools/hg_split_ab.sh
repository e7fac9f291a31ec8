#!/bin/bash
# c5 per-slot ms for several WST_HG_SPLIT settings (dev tool, GPU box, needs a -DWST_DIAG library)
# usage: tools/hg_split_ab.sh <lib> <split>...
cd "$GRAFT_REPO_ROOT" || exit 99
lib=$1; shift
for sp in "$@"; do
  WST_LIB=$lib WST_HG_SPLIT=$sp timeout -k 10 200 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/hgs.log 2>&1 || exit 9
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/hgs.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('split $sp', d['ms_per_step'], 'o2 j1=0', k['k_o2_j1=0'], 'j1=1', k['k_o2_j1=1'], 'o1 j1=0', k['k_o1_j1=0'])"
done
