#!/bin/bash
# A/B timing + LDS stall counters of library variants (dev tool). usage: tools/ab_libs.sh lib1.so lib2.so ...
out=gpurun_out/ab; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  AB_LIB=$lib timeout -k 10 200 python3 tools/kernel_ms.py > $out/$lib.time 2>&1 || { echo "time $lib failed"; tail -5 $out/$lib.time; exit 99; }
  AB_LIB=$lib timeout -k 10 200 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $out/${lib}_pmc -o pmc -- python3 tools/time_c2.py --iters 1 > $out/$lib.pmclog 2>&1 || { echo "pmc $lib failed"; exit 99; }
  echo "== $lib: $(tail -1 $out/$lib.time)"
  python3 tools/pmc_summary.py $out/${lib}_pmc 2>/dev/null | grep -E "==|UNALIGNED|IDX_ACTIVE|BANK|WAIT_ANY|WAVE_CYCLES" | grep -A5 "136\|prep" | head -14
done
