#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free box / slot (the call
# never started: status=transient, nothing charged). Any call that ran -- pass or fail -- ends the
# loop. Usage: scripts/gpurun_wait.sh <out-file> <timeout-s> '<command>'
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out" && ! grep -q "run [1-9]" "$out"; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
