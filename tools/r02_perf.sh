#!/bin/bash
# GPU parity tests (-x) then bench lines for the listed configs (no CPU baseline).
# usage: tools/r02_perf.sh <tag> <config>...
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread || exit 99
tail -4 gpurun_out/${tag}_pytest.txt
grep -q " passed" gpurun_out/${tag}_pytest.txt && ! grep -q "failed" gpurun_out/${tag}_pytest.txt || exit 98
for c in "$@"; do
  tools/gpu_step.sh 300 gpurun_out/${tag}_${c}_bench.log python3 bench.py --config $c --steps 10 --no-cpu-baseline || exit 99
  grep '^{"metric"' gpurun_out/${tag}_${c}_bench.log > gpurun_out/${tag}_${c}_bench.json
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/${tag}_${c}_bench.json')); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], r['kernel'], r['frac'], json.dumps(r['kernel_ms_per_step']), d.get('measured'))"
done
