#!/bin/bash
# A/B of library variants by rocprof kernel averages (dev): tools/ab_kernel.sh <tag> <regex> lib1.so lib2.so ...
# prints the average duration of every kernel whose name matches <regex>, per library
tag=$1; rx=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
for lib in "$@"; do
  d=gpurun_out/$tag/${lib%.so}
  AB_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/kernel_ms.py 1536 > $d.log 2>&1 || { echo "$lib failed"; tail -5 $d.log; exit 99; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 tools/kstats.py "$rx" "$f"
done
