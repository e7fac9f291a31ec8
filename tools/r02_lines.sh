#!/bin/bash
# Bench lines for the secondary configs (c3, c4, f3 pooled) at the current build.  usage: tools/r02_lines.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
for c in "c3" "c4" "f3 --pooled"; do
  set -- $c
  t=${tag}_$1$( [ -n "$2" ] && echo p )
  tools/gpu_step.sh 400 gpurun_out/${t}_bench.log python3 bench.py --config $c || exit 99
  grep '^{"metric"' gpurun_out/${t}_bench.log > gpurun_out/${t}_bench.json || exit 98
  python3 -c "import json; d=json.load(open('gpurun_out/${t}_bench.json')); print('$t', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
