#!/bin/bash
# Round-5 A/B: the s = 2 all-paths row pass with two planes per workgroup vs one (var_base)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
tools/gpu_step.sh 600 gpurun_out/r05x_pytest.txt python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/r05x_pytest.txt
bash tools/ab_rep.sh r05x5 256,256,6,12 2 libwst_hip.so var_base.so || exit 99
