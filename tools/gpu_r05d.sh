#!/bin/bash
# r05d: variant GPU tests on the new trace layout, then alternating A/B at c2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/r05d_variants.txt python3 -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread || exit 99
tail -2 gpurun_out/r05d_variants.txt
bash tools/ab_rep.sh r05d 3072,64,4 2 libwst_hip.so var_notrace.so var_r04.so var_fg3.so var_fg6.so
