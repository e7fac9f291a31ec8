#!/bin/bash
# FFT-split A/B (WST_SPLITnn build knobs): per variant a quick c2-geometry parity check, then c2
# per-kernel timing alternating default / variants over 3 rounds.  usage: tools/r03_split.sh <tag> <var.so>...
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
for v in "$@"; do
  WST_LIB=$v tools/gpu_step.sh 300 gpurun_out/$tag/pytest_$v.txt python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
      --timeout 120 --timeout-method thread -k "c2 or c5 or order1 or cmp or pooled or full_size" || exit 99
  echo "$v: $(tail -n 1 gpurun_out/$tag/pytest_$v.txt)"
done
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99
  for v in "$@"; do WST_LIB=$v timeout -k 10 120 python3 tools/kernel_ms.py 1536 || exit 99; done
done 2>&1 | grep chunk
