#!/bin/bash
# fa_bwd_hs.hip: causal mask only on the diagonal path vs compare + select on every tile (probe build)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fa_bwd_fused_gpu.py -x -q -k "hs or step_layout" --timeout 120 --timeout-method thread > gpurun_out/hs_tests4.log 2>&1 || { tail -30 gpurun_out/hs_tests4.log; exit 1; }
tail -1 gpurun_out/hs_tests4.log
FA_AB_SHAPES="96,25,512,64,1;24,25,512,64,1;8,16,1024,64,1" python scripts/ab.py fa "maskall:CS336_FA_BWD=3,CS336_LIB=cs336_systems/_native/variants/maskall/libcs336_hip.so" "diag:CS336_FA_BWD=3" --rounds 2 || exit 1
python scripts/ab.py bench "maskall:CS336_LIB=cs336_systems/_native/variants/maskall/libcs336_hip.so" "diag:" --rounds 2 --steps 10
