#!/bin/bash
# Round-2 check: GPU tests (all, no -x), default bench line, smoke.  usage: tools/r02_check.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -q -rs --timeout 120 --timeout-method thread || exit 99
tail -25 gpurun_out/${tag}_pytest.txt
tools/gpu_step.sh 300 gpurun_out/${tag}_bench.log python3 bench.py || exit 99
grep '^{"metric"' gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
tools/gpu_step.sh 200 gpurun_out/${tag}_smoke.txt python3 -c "import __graft_entry__ as g; g.smoke()" || exit 99
tail -2 gpurun_out/${tag}_smoke.txt
