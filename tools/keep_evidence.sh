#!/bin/bash
# Copy one session's round evidence from gpurun_out/ into profiles/ (committed):
#   tools/keep_evidence.sh <tag>
tag=$1; o=gpurun_out; p=profiles
for f in $o/${tag}_*bench.json $o/${tag}_*frac_check.json $o/${tag}_*kernel_stats.csv $o/${tag}_*kernel_trace.csv \
         $o/${tag}_pytest.txt $o/${tag}_smoke.txt; do
  [ -f "$f" ] && cp "$f" $p/
done
for f in $o/${tag}_pmc.json $o/${tag}_*_pmc.json; do
  [ -f "$f" ] || continue
  b=$(basename "$f" .json); b=${b%_pmc}; cp "$f" $p/pmc_${b}.json
done
[ -f $o/${tag}_sq.txt ] && cp $o/${tag}_sq.txt $p/${tag}_sq.txt
ls $p | grep -c "$tag"
