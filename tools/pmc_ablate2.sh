#!/bin/bash
# VALU / SALU / LDS instruction counts of the c2 kernels per WST_DEBUG_SKIP mask (dev tool).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
for m in 0 8 16 64 88; do
  out=gpurun_out/pmcab_$m
  WST_DEBUG_SKIP=$m timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES --output-format csv -d $out -o pmc -- python3 tools/time_c2.py --iters 1 > $out.log 2>&1 || { echo "fail $m"; tail $out.log; exit 99; }
  echo "== mask $m"; python3 tools/pmc_summary.py $out | grep -A8 "k_o2<3, 3, 136" | grep -E "VALU |SALU|LDS |INT32|WAVE_CYCLES"
done
