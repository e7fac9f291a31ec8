#!/bin/bash
# rocprofv3 kernel-trace stats + HBM PMC passes + bench line for one config (GPU box only).
# usage: tools/profile_cfg.sh <tag> <config> [bench args for the final line...]
#   -> gpurun_out/<tag>_<config>_{kernel_stats.csv,bench.json} and profiles/pmc_<tag>_<config>.json
tag=$1; cfg=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
o=gpurun_out
t=${tag}_${cfg}
mkdir -p $o
sha=$(python3 -c "import bench; print(bench.src_sha())")
tools/gpu_step.sh 300 $o/${t}_ktrace.log rocprofv3 --kernel-trace --stats --output-format csv -d $o/${t}_ktrace -o run -- python3 bench.py --config $cfg --steps 60 --warmup 5 --no-cpu-baseline --no-probes &&
tools/gpu_step.sh 300 $o/${t}_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${t}_fetch -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 &&
tools/gpu_step.sh 300 $o/${t}_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${t}_write -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-probes --profile-iters 1 &&
python3 tools/pmc_hbm.py $o/${t}_fetch $o/${t}_write "$sha" $o/${t}_pmc.json > /dev/null &&
cp $o/${t}_pmc.json profiles/pmc_${t}.json &&
find $o/${t}_ktrace -name "*kernel_stats.csv" -exec cp {} $o/${t}_kernel_stats.csv \; &&
find $o/${t}_ktrace -name "*kernel_trace.csv" -exec cp {} $o/${t}_kernel_trace.csv \; &&
tools/gpu_step.sh 400 $o/${t}_bench.log python3 bench.py --config $cfg "$@" &&
grep '^{"metric"' $o/${t}_bench.log > $o/${t}_bench.json &&
python3 tools/frac_check.py $o/${t}_bench.json $o/${t}_kernel_stats.csv $o/${t}_kernel_trace.csv 5 | tee $o/${t}_frac_check.json &&
python3 -c "
import json; d=json.load(open('$o/${t}_bench.json')); r=d['roofline']
print('$cfg', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['traffic'])" &&
echo "[profile_cfg] done $t sha=$sha"
