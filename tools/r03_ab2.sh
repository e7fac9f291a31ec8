#!/bin/bash
# c2 A/B of the default library against variants (alternating, 3 rounds) + quick parity: tools/r03_ab2.sh <tag> <var.so>...
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 300 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread || exit 99
tail -1 gpurun_out/$tag/pytest.txt
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99
  for v in "$@"; do WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99; done
done 2>&1 | grep chunk
