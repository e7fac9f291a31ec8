#!/bin/bash
# parity (c2-family GPU tests) + rocprof kernel stats of the c2 step.  usage: tools/r03_s5.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread || exit 99
tail -5 gpurun_out/$tag/pytest.txt
bash tools/r03_prof.sh $tag 1536 || exit 99
grep wall gpurun_out/$tag/prof.log
