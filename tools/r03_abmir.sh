#!/bin/bash
# c2 mirror-fold A/B + the whole GPU suite: tools/r03_abmir.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread || exit 99
tail -1 gpurun_out/$tag/pytest.txt
for r in 1 2 3; do
  for v in libwst_hip.so var_nomir.so; do WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99; done
done 2>&1 | grep chunk
