#!/bin/bash
# phase ablation (diag build) at f3 and c2: tools/r03_abl.sh <tag>
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
WST_KM_GEOM=768,128,2 tools/gpu_step.sh 400 gpurun_out/$tag/abl_f3.txt python3 tools/ablate.py || exit 99
cat gpurun_out/$tag/abl_f3.txt
tools/gpu_step.sh 400 gpurun_out/$tag/abl_c2.txt python3 tools/ablate.py || exit 99
cat gpurun_out/$tag/abl_c2.txt
