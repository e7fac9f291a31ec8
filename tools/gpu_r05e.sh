#!/bin/bash
# r05e: GPU tests (variant cover + full suite), c2 A/B (trace / fuse groups / round 4), c5 A/B, f3 split PMC
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/r05e_variants.txt python3 -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread || exit 99
tail -2 gpurun_out/r05e_variants.txt
tools/gpu_step.sh 600 gpurun_out/r05e_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 200 --timeout-method thread --deselect tests/test_gpu_variants.py || exit 99
tail -2 gpurun_out/r05e_pytest.txt
grep -q " passed" gpurun_out/r05e_pytest.txt || exit 99
bash tools/ab_rep.sh r05e 3072,64,4 2 libwst_hip.so var_notrace.so var_notslot.so var_r04.so || exit 99
bash tools/ab_rep.sh r05e5 256,256,6,12 1 libwst_hip.so var_r04.so || exit 99
bash tools/f3_split.sh r05e
