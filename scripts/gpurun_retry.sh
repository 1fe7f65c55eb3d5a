#!/bin/bash
# Runs one gpurun call; repeats it ONLY when gpurun reports an infrastructure
# event ("status=transient": box lost while being prepared / taken away; nothing
# ran, nothing charged).  Any run that actually executed is never repeated.
#   usage: scripts/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; lim=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "charged=[1-9]" "$log"; then
    echo "[retry $i: transient infrastructure event]" >> "$log.retries"
    sleep 45
    continue
  fi
  exit $rc
done
exit $rc
