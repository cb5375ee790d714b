#!/bin/bash
# Batch-102 GEMM report (table entries for 52224 tokens) + step profile, one GPU call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CS336_GEMM_REPORT=gpurun_out/rep102.json timeout -k 10 300 python -u bench.py --batch 102 --steps 2 --warmup 2 > gpurun_out/rep102.log 2>&1 || exit $?
tail -1 gpurun_out/rep102.log
PROF_TAG=_b102 BENCH_ARGS="--batch 102" ROOF_ARGS="--batch 102" bash scripts/prof_xl_step.sh || exit $?
head -40 gpurun_out/xl_roofline_b102.md
