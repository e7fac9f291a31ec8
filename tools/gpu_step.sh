#!/bin/bash
# Run one GPU step under a time limit; abort the whole session on crash/timeout/fault.
# usage: tools/gpu_step.sh <seconds> <logfile> <cmd...>
# exit status 0/1 (pass / ordinary test failure) lets the session continue; anything else stops it.
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" | tee -a "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[gpu_step] fatal status $rc -> stopping session"; tail -30 "$log"; exit 99
fi
exit 0
