#!/bin/bash
# banded low-pass A/B: GPU parity of the default build, then f3 / c1 per-kernel timing against
# variants, alternating, 3 rounds.  usage: tools/r03_band.sh <tag> <var.so>...
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread || exit 99
tail -n 2 gpurun_out/$tag/pytest.txt
for g in 768,128,2 3072,64,2; do
  for r in 1 2 3; do
    WST_KM_GEOM=$g timeout -k 10 120 python3 tools/kernel_ms.py || exit 99
    for v in "$@"; do WST_KM_GEOM=$g WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py || exit 99; done
  done 2>&1 | grep chunk
done
