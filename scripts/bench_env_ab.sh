#!/bin/bash
# Same-box A/B of bench.py under env settings: each arg is "label:ENV=V,ENV2=V2" (empty = default).
# usage: scripts/bench_env_ab.sh "base:" "nodyt:CS336_DYT=0" ... ; prints label and ms/step per run.
set -u
mkdir -p gpurun_out
STEPS=${AB_STEPS:-10}
for round in 1 2; do
  for spec in "$@"; do
    label="${spec%%:*}"; envs="${spec#*:}"
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 200 python bench.py --steps $STEPS --warmup 3 > gpurun_out/ab_${label}_$round.log 2>&1 ) || { echo "run $label failed"; tail -5 gpurun_out/ab_${label}_$round.log; exit 1; }
    ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${label}_$round.log | awk '{print $2}')
    echo "round $round $label ms_per_step=$ms"
  done
done
