#!/bin/bash
# Round-5 A/B: box threshold 1e-8 (was 1e-10) vs the previous library (var_base); GPU tests first
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
tools/gpu_step.sh 600 gpurun_out/r05o_pytest.txt python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/r05o_pytest.txt
bash tools/ab_rep.sh r05o5 256,256,6,12 2 libwst_hip.so var_base.so || exit 99
bash tools/ab_rep.sh r05o 3072,64,4 2 libwst_hip.so var_base.so || exit 99
bash tools/ab_rep.sh r05o3 768,128,2 2 libwst_hip.so var_base.so || exit 99
