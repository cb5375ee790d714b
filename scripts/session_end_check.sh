#!/bin/bash
# Driver-shaped checks after a default change: GEMM/bench GPU tests, the default bench (N=1, 20 steps,
# 5 warmup), a 2-rank one-GPU rehearsal (gloo) of the default DDP path, and a kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_lt_gemm_gpu.py tests/test_bench_contract.py -m gpu > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 bash scripts/rehearse_multirank.sh > gpurun_out/rehearse.log 2>&1 || { tail -30 gpurun_out/rehearse.log; exit 1; }
grep '"metric"' gpurun_out/rehearse.log | cut -c1-400
PROF_TAG=_final bash scripts/prof_xl_step.sh && head -40 gpurun_out/xl_roofline_final.md
