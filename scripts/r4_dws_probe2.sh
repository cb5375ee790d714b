#!/bin/bash
# Does the dW side-stream slowdown (profiles/r4_dw_stream.md) show without the profiler at 2 timed
# steps (it did not under rocprofv3 --kernel-trace), and does RCCL-shaped side work (resident
# channel workgroups / bucket copies) slow the XL step beyond the resources it takes?
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 240 "$@" 2>&1 | grep -E '^\{' ; }
run env CS336_DW_STREAM=1 python bench.py --batch 48 --steps 2 --warmup 2 &&
run env CS336_DW_STREAM=1 python bench.py --batch 48 --steps 10 --warmup 2 &&
run python bench.py --batch 48 --steps 10 --warmup 2 &&
run env CS336_DW_STREAM=1 HIP_LAUNCH_BLOCKING=0 AMD_SERIALIZE_KERNEL=0 GPU_MAX_HW_QUEUES=2 python bench.py --batch 48 --steps 10 --warmup 2 &&
echo "== side noise" && timeout -k 10 300 python scripts/r4_side_noise.py --batch 16
