#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/r03abprep
tools/gpu_step.sh 300 gpurun_out/r03abprep/pytest.txt python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_patterns.py -m gpu -q -x --timeout 120 --timeout-method thread || exit 99
tail -1 gpurun_out/r03abprep/pytest.txt
for r in 1 2; do
  for v in libwst_hip.so var_head17.so; do WST_KM_GEOM=768,128,2 WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 768 || exit 99; done
done 2>&1 | grep chunk
bash tools/r03_skip.sh 2>&1 | grep skip=
