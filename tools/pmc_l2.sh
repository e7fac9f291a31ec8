#!/bin/bash
# L2 (TCC) hit / miss per kernel for one config (dev tool, GPU box).  usage: tools/pmc_l2.sh <tag> <config>
tag=$1; cfg=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
o=gpurun_out/l2_$tag; mkdir -p $o
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $o -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 > $o/run.log 2>&1 || { tail -5 $o/run.log; exit 99; }
python3 - "$o" <<'PY'
import collections, csv, glob, sys, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("TCC_MISS_sum", 0)):
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    if h + m: print(f"{k[:70]:70s} hit {h:.3e} miss {m:.3e} hit-rate {h/(h+m):.1%}")
PY
