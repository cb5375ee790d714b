#!/bin/bash
# two-kernel FA2 backward: dQ and dK/dV kernels concurrently on two streams (CS336_FA_BWD_CONC=1) vs serial
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_flash_long_gpu.py -x -q -k "concurrent" --timeout 120 --timeout-method thread > gpurun_out/conc_tests.log 2>&1 || { tail -30 gpurun_out/conc_tests.log; exit 1; }
tail -1 gpurun_out/conc_tests.log
FA_AB_SHAPES="4,16,4096,64,1;4,16,4096,64,0;4,16,4096,128,1;4,16,4096,128,0;16,16,16384,64,1" python scripts/ab.py fa "serial:CS336_FA_BWD=0" "conc:CS336_FA_BWD=0,CS336_FA_BWD_CONC=1" --rounds 2
