#!/bin/bash
# One GPU session, parameterised (GPU box only; replaces the per-session gpu_rNN*.sh scripts):
#   tools/session.sh <tag> <step> [<step> ...]
# Steps run in order; each GPU step runs under its own time limit (tools/gpu_step.sh) and the
# session stops at the first fatal status (crash, abort, timeout).  Outputs: gpurun_out/<tag>_*.
#   pytest[=<file>]                     GPU tests (all of -m gpu, or one test file)
#   ab=<geom>:<reps>:<lib>[,<lib>...]   alternating per-kernel HIP-event A/B of library builds in the
#                                       package dir (tools/ab_rep.sh); geom = planes,M,J[,L]
#   env=<name>:<lib>:<geom>[:VAR=v+...] per-kernel ms of one library under env settings (diagnostic
#                                       builds read WST_* knobs)
#   km=<geom>:<chunk>[,<chunk>...][:<lib>]  per-kernel ms at several chunk sizes (planes per chunk)
#   abl=<geom>:<mask>[,<mask>...]      phase ablation (tools/ablate.py, diagnostic build libwst_hip_diag.so)
#   pat=<lib>[,<lib>...]               c5-geometry structured-pattern errors per build (tools/pattern_check.py)
#   sq=<geom>[:<lib>]                   SQ counter passes of one forward (tools/pmc.sh) -> <tag>_sq summary
#   evidence=<cfg>[,<cfg>...]           round evidence (tools/round_evidence.sh)
#   bench[=<arg>,<arg>...]              one bench.py line (no CPU baseline)
# example: tools/session.sh r06a pytest sq=3072,64,4 ab=3072,64,4:3:libwst_hip.so,var_base.so
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out
o=gpurun_out
for step in "$@"; do
  kind=${step%%=*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*=}
  echo "[session $tag] $step"
  case $kind in
    pytest)
      sel=${arg:-tests}; flt=""; [ -z "$arg" ] && flt="-m gpu"
      tools/gpu_step.sh 600 $o/${tag}_pytest.txt python3 -u -m pytest $sel $flt -x -q -rs --timeout 200 --timeout-method thread || exit 99
      tail -3 $o/${tag}_pytest.txt
      grep -qE "[0-9]+ passed" $o/${tag}_pytest.txt && ! grep -qE "[0-9]+ failed" $o/${tag}_pytest.txt || exit 99 ;;
    ab)
      IFS=: read -r geom reps libs <<< "$arg"
      bash tools/ab_rep.sh ${tag} $geom $reps ${libs//,/ } || exit 99 ;;
    env)
      IFS=: read -r name lib geom vars <<< "$arg"
      env ${vars//+/ } AB_LIB=$lib WST_KM_GEOM=$geom timeout -k 10 200 python3 tools/kernel_ms.py 1536 > $o/${tag}_$name.txt 2>&1 \
        || { echo "$name failed"; tail -3 $o/${tag}_$name.txt; exit 99; }
      echo "$name $(tail -1 $o/${tag}_$name.txt)" ;;
    km)
      IFS=: read -r geom chunks lib <<< "$arg"
      AB_LIB=$lib WST_KM_GEOM=$geom timeout -k 10 300 python3 tools/kernel_ms.py ${chunks//,/ } > $o/${tag}_km.txt 2>&1 \
        || { echo "km failed"; tail -3 $o/${tag}_km.txt; exit 99; }
      cat $o/${tag}_km.txt ;;
    abl)
      IFS=: read -r geom masks <<< "$arg"
      WST_KM_GEOM=$geom timeout -k 10 600 python3 tools/ablate.py ${masks//,/ } > $o/${tag}_abl.txt 2>&1 \
        || { echo "abl failed"; tail -3 $o/${tag}_abl.txt; exit 99; }
      cat $o/${tag}_abl.txt ;;
    pat)
      for lib in ${arg//,/ }; do
        AB_LIB=$lib timeout -k 10 200 python3 tools/pattern_check.py > $o/${tag}_pat_$lib.txt 2>&1 \
          || { echo "pat $lib failed"; tail -3 $o/${tag}_pat_$lib.txt; exit 99; }
        cat $o/${tag}_pat_$lib.txt
      done ;;
    sq)
      IFS=: read -r geom lib <<< "$arg"
      IFS=, read -r b m j l <<< "$geom"
      AB_LIB=$lib bash tools/pmc.sh ${tag}_sq python3 tools/time_c2.py --B $b --C 1 --M $m --J $j --L ${l:-8} --iters 1 || exit 99
      cp $o/pmc_${tag}_sq/summary.txt $o/${tag}_sq.txt ;;
    evidence)
      bash tools/round_evidence.sh $tag ${arg//,/ } || exit 99 ;;
    bench)
      tools/gpu_step.sh 300 $o/${tag}_bench.log python3 bench.py --no-cpu-baseline ${arg//,/ } || exit 99
      grep '^{"metric"' $o/${tag}_bench.log | tail -1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[session $tag] done"
