#!/bin/bash
# round-end evidence, part 2: f3 / c1 / c5 profiles, f3-pooled / c3 / c4 bench lines
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
bash tools/profile_cfg.sh $tag f3 || exit 99
bash tools/profile_cfg.sh $tag c1 || exit 99
bash tools/profile_cfg.sh $tag c5 || exit 99
tools/gpu_step.sh 300 gpurun_out/${tag}_f3p_bench.log python3 bench.py --config f3 --pooled || exit 99
grep '^{"metric"' gpurun_out/${tag}_f3p_bench.log > gpurun_out/${tag}_f3p_bench.json
tools/gpu_step.sh 400 gpurun_out/${tag}_c3_bench.log python3 bench.py --config c3 || exit 99
grep '^{"metric"' gpurun_out/${tag}_c3_bench.log > gpurun_out/${tag}_c3_bench.json
tools/gpu_step.sh 300 gpurun_out/${tag}_c4_bench.log python3 bench.py --config c4 || exit 99
grep '^{"metric"' gpurun_out/${tag}_c4_bench.log > gpurun_out/${tag}_c4_bench.json
echo done
