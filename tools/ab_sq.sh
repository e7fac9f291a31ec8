#!/bin/bash
# A/B of k_o2 phases on the square fused path (dev tool): per env setting, per-kernel ms.
cd "$GRAFT_REPO_ROOT" || exit 99
for e in "WST_SQ=1" "WST_BOX=0" "WST_DEBUG_SKIP=8" "WST_DEBUG_SKIP=16" "WST_DEBUG_SKIP=64" "WST_DEBUG_SKIP=88" "WST_DEBUG_SKIP=4"; do
  env $e timeout -k 10 200 python3 tools/kernel_ms.py > gpurun_out/ab.tmp 2>&1 || { echo "failed: $e"; tail -5 gpurun_out/ab.tmp; exit 99; }
  echo "$e :: $(grep chunk gpurun_out/ab.tmp)"
done
