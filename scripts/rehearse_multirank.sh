#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE GPU (the driver runs the real 1/2/4/8-GPU RCCL bench):
# 2 ranks share cuda:0, gradients all-reduced over gloo (GPU tensors staged through the host),
# exercising DDP bucketing/hooks, the dW-into-bucket path, ZeRO-1 and the MAX-over-ranks timing.
# usage: scripts/rehearse_multirank.sh [extra bench.py args]
set -e
export CS336_DIST_BACKEND=gloo
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --batch 8 "$@"
