#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time limit and the script
# stops at the first crash-like exit (fault/abort/segv/timeout) so nothing else touches a sick GPU.
# usage: scripts/gpu_run.sh "name:timeout:command" ...
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${tmo}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -ge 128 ]; then
    echo "fatal exit code $rc in step $name; stopping"
    exit $rc
  fi
done
