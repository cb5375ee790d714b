#!/bin/bash
# FA2 A/B probes (round 4): key-block-parallel backward with / without its dQ atomics (a wrong-dQ
# timing probe built as a library variant), then the B 1 H 1 reference sweep (bf16) with the
# split-KV forward and split backward. Each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 200 env CS336_FA_BWD=2 python -u scripts/fa_ab.py > gpurun_out/r4/fa_ab_kp.log 2>&1 || exit $?
timeout -k 10 200 env CS336_FA_BWD=2 CS336_LIB=cs336_systems/_native/variants/noatom/libcs336_hip.so \
  python -u scripts/fa_ab.py > gpurun_out/r4/fa_ab_kp_noatom.log 2>&1 || exit $?
timeout -k 10 200 env CS336_FA_BWD=0 python -u scripts/fa_ab.py > gpurun_out/r4/fa_ab_two.log 2>&1 || exit $?
timeout -k 10 700 python -u -m cs336_systems.bench.flash --sweep --sweep-dtype bf16 \
  --json gpurun_out/r4/flash_sweep_bf16.json > gpurun_out/r4/flash_sweep_bf16.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/rehearse_multirank.sh --batch 8 --comm-sweep-mb 1 10 > gpurun_out/r4/rh_xl.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/rehearse_multirank.sh --model small --ctx 512 --batch 8 --ddp-sweep on --comm-sweep-mb 1 > gpurun_out/r4/rh_small_sweep.log 2>&1 || exit $?
