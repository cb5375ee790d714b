#!/bin/bash
# 2.7b per-GPU batch 24 vs 32 (ctx 1024), same box; the batch-32 GEMM problems timed at runtime and reported
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
CS336_GEMM_REPORT=gpurun_out/gemm_report_2p7b_b32.json timeout -k 10 400 python bench.py --model 2.7b --ctx 1024 --batch 32 --steps 8 --warmup 4 > gpurun_out/b2p7_32a.json 2> gpurun_out/b2p7_32a.err || { tail -20 gpurun_out/b2p7_32a.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' gpurun_out/b2p7_32a.json | tr '\n' ' '; echo
python scripts/ab.py bench "b24::--batch 24" "b32::--batch 32" --rounds 2 --steps 8 --args "--model 2.7b --ctx 1024"
