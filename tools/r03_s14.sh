#!/bin/bash
# parity (all GPU tests) + c5 / c2 bench lines: tools/r03_s14.sh <tag>
tag=$1
cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 900 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -v -rs --timeout 200 --timeout-method thread || exit 99
grep -E "passed|failed|FAILED|SKIPPED" gpurun_out/$tag/pytest.txt | tail -25
tools/gpu_step.sh 300 gpurun_out/$tag/bench_c5.json python3 bench.py --config c5 --steps 5 --warmup 2 || exit 99
tools/gpu_step.sh 300 gpurun_out/$tag/bench_c2.json python3 bench.py --steps 20 --warmup 5 || exit 99
tail -c 600 gpurun_out/$tag/bench_c5.json
