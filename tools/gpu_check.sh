#!/bin/bash
# GPU parity tests + per-kernel timing of the current build (dev tool): tools/gpu_check.sh <tag> [env settings for ab_env...]
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread || exit 99
tail -3 gpurun_out/${tag}_pytest.txt
bash tools/ab_env.sh "WST_DEBUG_SKIP=0" "$@"
