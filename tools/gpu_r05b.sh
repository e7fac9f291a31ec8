cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
tools/gpu_step.sh 500 gpurun_out/r05b_variants.txt python3 -u -m pytest tests/test_gpu_variants.py -x -q -rs --timeout 120 --timeout-method thread --durations=10 || exit 99
tail -15 gpurun_out/r05b_variants.txt
tools/gpu_step.sh 600 gpurun_out/r05b_pytest.txt python3 -u -m pytest tests -m gpu -x -q -rs --timeout 200 --timeout-method thread --deselect tests/test_gpu_variants.py || exit 99
tail -3 gpurun_out/r05b_pytest.txt
tools/gpu_step.sh 300 gpurun_out/r05b_bench.log python3 bench.py --no-cpu-baseline || exit 99
grep '^{"metric"' gpurun_out/r05b_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms_per_step'])"
