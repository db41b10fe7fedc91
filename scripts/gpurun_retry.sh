#!/bin/bash
# usage: scripts/gpurun_retry.sh <timeout> <command...>; retries transient infra failures (rc 3 / transient)
to=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  out=$(timeout $((to + 600)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" 2>&1)
  echo "$out" | tail -60
  if echo "$out" | grep -q "status=transient\|backing off\|rc=3 "; then sleep 120; continue; fi
  break
done
