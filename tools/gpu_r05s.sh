#!/bin/bash
# Round-5 A/B: HG k_o2 one workgroup per item (split 1) vs 4 (var_base); GPU tests first
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
tools/gpu_step.sh 600 gpurun_out/r05s_pytest.txt python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/r05s_pytest.txt
bash tools/ab_rep.sh r05s5 256,256,6,12 2 libwst_hip.so var_base.so || exit 99
