#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time
# limit.  A step that fails normally (exit 1: a test failure) lets the next
# step run; a fault / abort / segfault / timeout (any other non-zero code)
# ends the session immediately.
#   usage: scripts/gpu_session.sh "<limit_s> <cmd>" ...
mkdir -p gpurun_out
n=0
for spec in "$@"; do
  n=$((n+1))
  lim=${spec%% *}; cmd=${spec#* }
  echo "=== step $n (limit ${lim}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/step$n.log" 2>&1
  rc=$?
  echo "=== step $n rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/step$n.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
