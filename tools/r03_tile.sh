#!/bin/bash
# column-tiled staged round trip A/B: staged GPU parity, then c5 ms/step against variants (2 rounds)
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 500 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -x -q -rs --timeout 120 --timeout-method thread || exit 99
tail -n 1 gpurun_out/$tag/pytest.txt
for r in 1 2; do
  for v in libwst_hip.so "$@"; do
    WST_LIB=$v timeout -k 10 200 python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/$tag/c5_$v.$r.log 2>&1 || exit 99
    python3 -c "
import json,sys; d=[json.loads(l) for l in open('gpurun_out/$tag/c5_$v.$r.log') if l.startswith('{\"metric')][0]
print('$v', d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
  done
done
