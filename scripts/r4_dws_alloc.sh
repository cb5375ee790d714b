#!/bin/bash
# Allocator stats of the dW side-stream step (CS336_DW_STREAM=1) at batch 48: the record_stream form
# (CS336_DW_HOLD=0) at 2 / 10 timed steps and with a host sync per step (CS336_BENCH_SYNC_EACH=1
# caps the host's run-ahead at one step), vs holding dY / X with a bounded lag (default), vs base.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 240 "$@" 2>&1 | grep -E 'allocator:|^\{' | cut -c1-200 ; }
run env CS336_DW_STREAM=1 CS336_DW_HOLD=0 python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_DW_STREAM=1 CS336_DW_HOLD=0 CS336_BENCH_SYNC_EACH=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_DW_STREAM=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_DW_STREAM=1 python bench.py --steps 10 --warmup 2 &&
run python bench.py --steps 10 --warmup 2 &&
echo "== tests" && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dw_stream_gpu.py 2>&1 | tail -3
