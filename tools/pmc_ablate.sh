#!/bin/bash
# SQ_LDS_UNALIGNED_STALL per ablation mask (dev tool)
out=gpurun_out/pmc_abl; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 0 1 2 4 8 16 64 128 223; do
  WST_DEBUG_SKIP=$m timeout -k 10 200 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $out/m$m -o pmc -- python3 tools/time_c2.py --iters 1 > $out/m$m.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "mask $m rc=$rc"; tail -5 $out/m$m.log; exit 99; fi
  python3 - $out/m$m $m <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_order12<3, 3, 136>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
print("mask", sys.argv[2], {k: f"{v:.3e}" for k, v in sorted(agg.items())})
PY
done
