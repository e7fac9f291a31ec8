#!/bin/bash
# Per-slot ms of one config under several environment settings (dev tool, GPU box).
# usage: tools/env_ab.sh <lib> <config> "VAR=a VAR2=b" "VAR=c" ...
cd "$GRAFT_REPO_ROOT" || exit 99
lib=$1; cfg=$2; shift 2
for st in "$@"; do
  env WST_LIB=$lib $st timeout -k 10 200 python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 2 > gpurun_out/envab.log 2>&1 || { tail -5 gpurun_out/envab.log; exit 9; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/envab.log') if l.startswith('{')][-1]); k=d['roofline']['kernel_ms_per_step']
print('[$st]', d['ms_per_step'], {a: round(b, 3) for a, b in k.items() if b > 0.3})"
done
