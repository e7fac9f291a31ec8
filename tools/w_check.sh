#!/bin/bash
# Dev loop on the GPU box: c2 per-kernel timing, then the GPU tests (stop at the first failure).
# usage: tools/w_check.sh <tag> [pytest -k expr]
tag=$1; k=${2:-}
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 150 gpurun_out/${tag}_km.txt python3 tools/kernel_ms.py || exit 99
tail -1 gpurun_out/${tag}_km.txt
if [ -n "$k" ]; then
  tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread -k "$k" || exit 99
else
  tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread || exit 99
fi
tail -3 gpurun_out/${tag}_pytest.txt
