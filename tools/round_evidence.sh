#!/bin/bash
# Round-end evidence at the current source hash (GPU box only), one parametrised driver:
#   tools/round_evidence.sh <tag> [configs...]     default configs: c2 f3 c1 c5
# c2 -> tools/profile_round.sh (GPU tests first, then kernel stats + PMC + bench line + smoke);
# every other config -> tools/profile_cfg.sh; "f3p" / "c3" / "c4" -> bench lines only.
tag=$1; shift
cfgs=${@:-c2 f3 c1 c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
for c in $cfgs; do
  case $c in
    c2) tools/gpu_step.sh 600 gpurun_out/${tag}_pytest.txt python3 -u -m pytest tests -m gpu -v -rs --timeout 200 --timeout-method thread || exit 99
        tail -2 gpurun_out/${tag}_pytest.txt
        bash tools/profile_round.sh $tag || exit 99 ;;
    f3p) tools/gpu_step.sh 300 gpurun_out/${tag}_f3p_bench.log python3 bench.py --config f3 --pooled || exit 99
         grep '^{"metric"' gpurun_out/${tag}_f3p_bench.log > gpurun_out/${tag}_f3p_bench.json ;;
    c3|c4) tools/gpu_step.sh 400 gpurun_out/${tag}_${c}_bench.log python3 bench.py --config $c || exit 99
           grep '^{"metric"' gpurun_out/${tag}_${c}_bench.log > gpurun_out/${tag}_${c}_bench.json ;;
    *) bash tools/profile_cfg.sh $tag $c || exit 99 ;;
  esac
done
echo "[round_evidence] done $tag"
