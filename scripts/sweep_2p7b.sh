#!/bin/bash
# 2.7b ctx 1024 step on one box: per-GPU batch x GEMM selection
set -o pipefail
mkdir -p gpurun_out
for spec in "12 blas" "12 best" "24 best" "36 best"; do
  set -- $spec
  timeout -k 10 300 python bench.py --model 2.7b --ctx 1024 --batch $1 --gemm $2 --steps 6 --warmup 3 > gpurun_out/s27_$1_$2.json 2> gpurun_out/s27_$1_$2.err || { tail -5 gpurun_out/s27_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s27_$1_$2.json'));print('$1 $2', d['value'], d['ms_per_step'], d['peak_mem_gib'])"
done
