#!/bin/bash
# staged tests + goldens: tools/r03_s15.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -v -rs --timeout 200 --timeout-method thread || exit 99
grep -E "passed|failed|FAILED|Error|SKIPPED" gpurun_out/$tag/pytest.txt | tail -25
