#!/bin/bash
# Same-box A/B of FA2 backward forms at one shape (bench.flash, two interleaved rounds):
# the two-kernel form and the fused kernel's variants (CS336_FA_FUSED_VAR bits: 1 batched reads,
# 2 dQ split over 8 waves).   SHAPE="--seq 512 --batch 48 --heads 25 --d 64" scripts/fa_bwd_var_ab.sh
set -u
SHAPE=${SHAPE:---seq 512 --batch 48 --heads 25 --d 64}
for round in 1 2; do
  for spec in "two:CS336_FA_BWD=0" "v0:CS336_FA_BWD=1 CS336_FA_FUSED_VAR=0" "v1:CS336_FA_BWD=1 CS336_FA_FUSED_VAR=1" \
              "v2:CS336_FA_BWD=1 CS336_FA_FUSED_VAR=2" "v3:CS336_FA_BWD=1 CS336_FA_FUSED_VAR=3"; do
    label="${spec%%:*}"
    out=$(env ${spec#*:} timeout -k 10 120 python -m cs336_systems.bench.flash $SHAPE --causal 1 --impls hip_fa2 --rep 50 2>/dev/null | tail -1) || { echo "$label failed"; exit 1; }
    echo "round $round $label $(echo "$out" | grep -o '"bwd_ms": [0-9.]*') $(echo "$out" | grep -o '"bwd_tflops": [0-9.]*')"
  done
done
