#!/bin/bash
# rocprofv3 PC sampling of one short run (GPU box; dev tool): tools/pcsample.sh <tag> [cmd...]
# stochastic (hardware, with stall reasons) first; host_trap if the device refuses it.  A timeout or
# crash ends the script (no further GPU step).
tag=$1; shift
cmd=${@:-python3 tools/time_c2.py --iters 3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
out=gpurun_out/pcs_$tag; mkdir -p $out
for m in "stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576" "host_trap --pc-sampling-unit time --pc-sampling-interval 1"; do
  timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $m --output-format csv -d $out/${m%% *} -o pcs -- $cmd > $out/${m%% *}.log 2>&1
  rc=$?
  echo "[pcs] ${m%% *} rc=$rc"
  if [ $rc -eq 0 ]; then exit 0; fi
  if [ $rc -ge 124 ]; then tail -5 $out/${m%% *}.log; exit 99; fi
  tail -3 $out/${m%% *}.log
done
exit 1
