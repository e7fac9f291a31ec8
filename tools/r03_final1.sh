#!/bin/bash
# round-end evidence, part 1: full GPU tests, smoke, c2 profile (kernel stats + PMC + bench line)
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -v -rs --timeout 200 --timeout-method thread || exit 99
tail -2 gpurun_out/${tag}_pytest.txt
bash tools/profile_round.sh $tag || exit 99
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench.json')); r=d['roofline']
print('c2', d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['hbm_frac'])"
tail -3 gpurun_out/${tag}_smoke.txt
