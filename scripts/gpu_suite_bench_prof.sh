#!/bin/bash
# One gpurun call: full GPU test suite, the driver-shaped XL bench, the 2.7b ctx-1024 bench and a
# rocprofv3 kernel trace of the XL step (roofline + step sequence). Every GPU step has its own limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_xl.json 2> gpurun_out/bench_xl.err || { tail -20 gpurun_out/bench_xl.err; exit 1; }
cat gpurun_out/bench_xl.json
timeout -k 10 300 python bench.py --model 2.7b --ctx 1024 --batch 12 --steps 10 --warmup 3 > gpurun_out/bench_2p7b.json 2> gpurun_out/bench_2p7b.err || { tail -20 gpurun_out/bench_2p7b.err; exit 1; }
cat gpurun_out/bench_2p7b.json
bash scripts/prof_xl_step.sh && head -16 gpurun_out/xl_roofline.md
