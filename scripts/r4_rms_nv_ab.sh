#!/bin/bash
# RMSNorm NV 10/12 register fit (d_model 2560): GPU tests, then the 2.7b step A/B against the NV-16 rounding
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_add_rmsnorm_gpu.py tests/test_kernels_gpu.py -x -q -k "rmsnorm" --timeout 120 --timeout-method thread > gpurun_out/rms_tests.log 2>&1 || { tail -30 gpurun_out/rms_tests.log; exit 1; }
tail -1 gpurun_out/rms_tests.log
python scripts/ab.py bench "nv16:CS336_LIB=cs336_systems/_native/variants/nv16/libcs336_hip.so" "nv10:" --rounds 2 --steps 8 --args "--model 2.7b --ctx 1024"
