#!/bin/bash
# Round-5 A/B: S1 tap low-pass loops unrolled vs the previous library (var_base); GPU tests first
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
tools/gpu_step.sh 600 gpurun_out/r05aa_pytest.txt python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/r05aa_pytest.txt
bash tools/ab_rep.sh r05aa 3072,64,4 3 libwst_hip.so var_base.so || exit 99
