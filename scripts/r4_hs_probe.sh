#!/bin/bash
# fa_bwd_hs.hip (two 4-wave workgroups per CU): GPU numerics, then same-box A/B against the fused
# head-sequential kernel (kernel timing on the step's shapes, then the XL step).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fa_bwd_fused_gpu.py -x -q -k "hs" --timeout 120 --timeout-method thread > gpurun_out/hs_tests.log 2>&1 || { tail -30 gpurun_out/hs_tests.log; exit 1; }
tail -1 gpurun_out/hs_tests.log
export FA_AB_SHAPES="96,25,512,64,1;24,25,512,64,1;8,16,2048,64,1;8,16,1024,64,0"
python scripts/ab.py fa "fused:CS336_FA_BWD=1" "hs:CS336_FA_BWD=3" --rounds 2 || exit 1
[ "${HS_BENCH:-1}" = 1 ] || exit 0
python scripts/ab.py bench "fused:CS336_FA_BWD=1" "hs:CS336_FA_BWD=3" "hsr0:CS336_FA_BWD=3,CS336_FA_HS_ROPE=0" --rounds 2 --steps 10
