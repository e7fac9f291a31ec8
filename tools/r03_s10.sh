#!/bin/bash
# parity + c2 kernel stats (dev): tools/r03_s10.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread || exit 99
tail -3 gpurun_out/$tag/pytest.txt
timeout -k 10 200 python3 tools/kernel_ms.py 1536 2048 > gpurun_out/$tag/kms.txt 2>&1 || exit 99
grep chunk gpurun_out/$tag/kms.txt
bash tools/ab_kernel.sh $tag "k_o2r|k_o2<|k_o1<3, 3, 136" libwst_hip.so
