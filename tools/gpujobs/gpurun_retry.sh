#!/bin/bash
# Submit one gpurun call; while the pool reports no free box (rc 3: nothing ran, nothing
# charged), wait as long as gpurun asks (or 120 s) and submit again, at most 30 times.
# Any other outcome ends it.
#   bash tools/gpujobs/gpurun_retry.sh <log> <timeout s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "gpurun rc=$rc (try $i)" >> "$log"
  [ $rc -eq 3 ] || exit $rc
  wait_s=$(grep -o "retry in [0-9]*s" "$log" | tail -1 | grep -o "[0-9]*")
  sleep $(( ${wait_s:-120} + 15 ))
done
exit 3
