#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/r05f_variants.txt python3 -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread || exit 99
tail -1 gpurun_out/r05f_variants.txt
bash tools/ab_rep.sh r05f 3072,64,4 3 libwst_hip.so var_r04.so || exit 99
bash tools/ab_rep.sh r05f3 768,128,2 2 libwst_hip.so var_r04.so || exit 99
