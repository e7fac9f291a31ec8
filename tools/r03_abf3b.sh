#!/bin/bash
# f3 / c1 A/B against the previous commit's family objects + parity: tools/r03_abf3b.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 300 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_patterns.py -m gpu -q -x --timeout 120 --timeout-method thread || exit 99
tail -1 gpurun_out/$tag/pytest.txt
for r in 1 2; do
  for v in libwst_hip.so var_head17.so; do WST_KM_GEOM=768,128,2 WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 768 || exit 99; done
  for v in libwst_hip.so var_head9.so; do WST_KM_GEOM=3072,64,2 WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99; done
done 2>&1 | grep chunk
