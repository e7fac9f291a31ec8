#!/bin/bash
# Round-5 A/B: typed global / LDS store and tap pointers (no flat memory ops) vs the r05h library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
bash tools/ab_rep.sh r05j 3072,64,4 3 libwst_hip.so var_base.so || exit 99
bash tools/ab_rep.sh r05j3 768,128,2 2 libwst_hip.so var_base.so || exit 99
bash tools/ab_rep.sh r05j5 256,256,6,12 2 libwst_hip.so var_base.so || exit 99
tools/gpu_step.sh 600 gpurun_out/r05j_pytest.txt python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/r05j_pytest.txt
