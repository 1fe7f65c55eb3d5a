#!/bin/bash
# Runs one gpurun call; repeats it ONLY when gpurun reports an infrastructure
# event ("status=transient": box lost while being prepared / taken away, or
# the pool backing off; nothing ran, nothing charged), waiting out any
# announced back-off.  Any run that actually executed is never repeated.
#   usage: scripts/gpurun_retry.sh LOG TIMEOUT 'command' [TRIES]
log=$1; lim=$2; cmd=$3; tries=${4:-12}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "charged=[1-9]" "$log"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    wait_s=${wait_s:-45}
    echo "[retry $i: transient infrastructure event, waiting $((wait_s + 15))s]" >> "$log.retries"
    sleep $((wait_s + 15))
    continue
  fi
  exit $rc
done
exit $rc
