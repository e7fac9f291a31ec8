#!/bin/bash
# round-end evidence at the current source hash: GPU tests, smoke, c2 + f3 + c1 + c5 profiles and bench lines
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -v -rs --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/${tag}_pytest.txt
bash tools/profile_round.sh $tag || exit 99
bash tools/profile_cfg.sh $tag f3 || exit 99
bash tools/profile_cfg.sh $tag c1 || exit 99
bash tools/profile_cfg.sh $tag c5 || exit 99
tools/gpu_step.sh 300 gpurun_out/${tag}_f3p_bench.log python3 bench.py --config f3 --pooled || exit 99
grep '^{"metric"' gpurun_out/${tag}_f3p_bench.log > gpurun_out/${tag}_f3p_bench.json
echo done
