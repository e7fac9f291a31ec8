#!/bin/bash
# rocprofv3 kernel stats of one config's bench (dev): tools/r03_prof.sh <tag> [bench args...]
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/prof -o run -- python3 tools/kernel_ms.py "$@" > gpurun_out/$tag/prof.log 2>&1 || { tail -20 gpurun_out/$tag/prof.log; exit 99; }
f=$(find gpurun_out/$tag/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/$tag/kernel_stats.csv
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms  n={r['Calls']:>5}  avg={float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
