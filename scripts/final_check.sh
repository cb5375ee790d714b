#!/bin/bash
# End-of-session: full GPU suite, default bench (driver shape), FA seq-4096 table, 2.7b step
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python -m cs336_systems.bench.flash --impls hip_fa2 --no-compile --json gpurun_out/flash4096.json > gpurun_out/flash4096.log 2>&1 || { tail gpurun_out/flash4096.log; exit 1; }
timeout -k 10 300 python -m cs336_systems.bench.flash --leaderboard --impls hip_fa2 --no-compile --json gpurun_out/flash_leaderboard.json > gpurun_out/flash_lb.log 2>&1 || { tail gpurun_out/flash_lb.log; exit 1; }
python - <<'P'
import json
for r in json.load(open('gpurun_out/flash4096.json')):
    print(r['impl'], r['N'], r['d'], r['causal'], 'fwd', round(r['fwd_tflops']), 'bwd', round(r['bwd_tflops']))
print(json.load(open('gpurun_out/flash_leaderboard.json')))
P
timeout -k 10 300 python bench.py --model 2.7b --ctx 1024 --batch 12 --steps 10 --warmup 3 > gpurun_out/bench_2p7b.json 2> gpurun_out/bench_2p7b.err || { tail -20 gpurun_out/bench_2p7b.err; exit 1; }
cut -c1-200 gpurun_out/bench_2p7b.json
