#!/bin/bash
# c5 A/B of library variants (alternating, 2 passes): tools/r03_c5ab.sh <tag> <var.so>...
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
for pass in 1 2; do
for v in libwst_hip.so "$@"; do
  WST_LIB=$v timeout -k 10 200 python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/$tag/b.log 2>&1 || exit 9
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$tag/b.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('pass $pass $v', d['ms_per_step'], {a: round(b, 3) for a, b in k.items() if b > 0.5})"
done
done
