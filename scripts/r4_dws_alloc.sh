#!/bin/bash
# Allocator stats of the dW side-stream step (CS336_DW_STREAM=1): 2 vs 10 timed steps, and 10 steps
# with a host sync per step (CS336_BENCH_SYNC_EACH=1 caps the host's run-ahead at one step).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 240 "$@" 2>&1 | grep -E 'allocator:|^\{' | cut -c1-200 ; }
run env CS336_DW_STREAM=1 python bench.py --batch 48 --steps 2 --warmup 2 &&
run env CS336_DW_STREAM=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_DW_STREAM=1 CS336_BENCH_SYNC_EACH=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_BENCH_SYNC_EACH=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run python bench.py --batch 48 --steps 10 --warmup 2
