#!/bin/bash
# dW GEMMs (gemm8w) on the side stream: GPU tests, then same-box A/B of the XL step
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dw_stream_gpu.py tests/test_concurrency_gpu.py tests/test_opt_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dws_tests.log 2>&1 || { tail -30 gpurun_out/dws_tests.log; exit 1; }
tail -1 gpurun_out/dws_tests.log
python scripts/ab.py bench "base:" "dws:CS336_DW_STREAM=1" --rounds 2 --steps 10
