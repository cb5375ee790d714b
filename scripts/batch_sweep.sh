#!/bin/bash
# XL per-GPU batch sweep on one box (bench.py, ctx 512): tokens/s per batch size
set -o pipefail
mkdir -p gpurun_out
for b in ${BATCHES:-24 32 40 48}; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/bsweep_$b.json 2> gpurun_out/bsweep_$b.err || { tail -5 gpurun_out/bsweep_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bsweep_$b.json'));print($b, d['value'], d['ms_per_step'], d['peak_mem_gib'])"
done
