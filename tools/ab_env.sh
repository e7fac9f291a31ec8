#!/bin/bash
# A/B kernel timings across env settings (dev tool): tools/ab_env.sh "VAR=val ..." "VAR=val ..." ...
cd "$GRAFT_REPO_ROOT" || exit 99
for e in "$@"; do
  env $e timeout -k 10 200 python3 tools/kernel_ms.py > gpurun_out/ab_env.tmp 2>&1 || { echo "failed: $e"; tail -5 gpurun_out/ab_env.tmp; exit 99; }
  echo "$e :: $(grep chunk gpurun_out/ab_env.tmp)"
done
