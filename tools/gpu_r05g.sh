#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/r05g_variants.txt python3 -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread || exit 99
tail -3 gpurun_out/r05g_variants.txt
grep -q " passed" gpurun_out/r05g_variants.txt || exit 99
bash tools/ab_rep.sh r05g 3072,64,4 3 libwst_hip.so var_r04.so || exit 99
bash tools/ab_rep.sh r05g3 768,128,2 2 libwst_hip.so var_r04.so || exit 99
