#!/bin/bash
# Round-3 session: GPU parity + per-kernel timing of the c2 step.  usage: tools/r03_s2.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread || exit 99
tail -15 gpurun_out/$tag/pytest.txt
tools/gpu_step.sh 300 gpurun_out/$tag/kms.txt python3 tools/kernel_ms.py 1536 2048 || exit 99
cat gpurun_out/$tag/kms.txt
