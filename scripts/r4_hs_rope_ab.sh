set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fa_bwd_fused_gpu.py -x -q -k "hs or step_layout" --timeout 120 --timeout-method thread > gpurun_out/hs_tests2.log 2>&1 || { tail -30 gpurun_out/hs_tests2.log; exit 1; }
tail -1 gpurun_out/hs_tests2.log
python scripts/ab.py bench "r0:" "r2:CS336_FA_HS_ROPE=2" --rounds 3 --steps 10
# probe: the hs kernel without its dQ partial loads (wrong dQ; timing only)
FA_AB_SHAPES="96,25,512,64,1;24,25,512,64,1" python scripts/ab.py fa "hs:CS336_FA_BWD=3" "nopp:CS336_FA_BWD=3,CS336_LIB=cs336_systems/_native/variants/nopp/libcs336_hip.so" --rounds 2
