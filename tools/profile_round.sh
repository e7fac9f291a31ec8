#!/bin/bash
# rocprofv3 kernel-trace stats + HBM PMC passes for one library build, then the bench line (which
# picks up the PMC traffic of this source hash from profiles/).  GPU box only.
# usage: tools/profile_round.sh <tag>    -> gpurun_out/<tag>_*  (copy summaries into profiles/)
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
o=gpurun_out
mkdir -p $o
sha=$(python3 -c "import bench; print(bench.src_sha())")
tools/gpu_step.sh 300 $o/${tag}_ktrace.log rocprofv3 --kernel-trace --stats --output-format csv -d $o/${tag}_ktrace -o run -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline &&
tools/gpu_step.sh 300 $o/${tag}_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${tag}_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 &&
tools/gpu_step.sh 300 $o/${tag}_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${tag}_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 &&
python3 tools/pmc_hbm.py $o/${tag}_fetch $o/${tag}_write "$sha" $o/${tag}_pmc.json > /dev/null &&
cp $o/${tag}_pmc.json profiles/pmc_${tag}.json &&
find $o/${tag}_ktrace -name "*kernel_stats.csv" -exec cp {} $o/${tag}_kernel_stats.csv \; &&
find $o/${tag}_ktrace -name "*kernel_trace.csv" -exec cp {} $o/${tag}_kernel_trace.csv \; &&
tools/gpu_step.sh 400 $o/${tag}_bench.log python3 bench.py &&
grep '^{"metric"' $o/${tag}_bench.log > $o/${tag}_bench.json &&
python3 tools/frac_check.py $o/${tag}_bench.json $o/${tag}_kernel_stats.csv $o/${tag}_kernel_trace.csv 5 | tee $o/${tag}_frac_check.json &&
tools/gpu_step.sh 200 $o/${tag}_smoke.txt python3 -c "import __graft_entry__ as g; g.smoke()" &&
echo "[profile_round] done $tag sha=$sha"
