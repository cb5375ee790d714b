#!/bin/bash
# fa_bwd_hs.hip with s_setprio(1) around its MFMA clusters (probe build) vs without
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
L=cs336_systems/_native/variants/prio/libcs336_hip.so
FA_AB_SHAPES="96,25,512,64,1;24,25,512,64,1" python scripts/ab.py fa "base:CS336_FA_BWD=3" "prio:CS336_FA_BWD=3,CS336_LIB=$L" --rounds 2 || exit 1
python scripts/ab.py bench "base:" "prio:CS336_LIB=$L" --rounds 2 --steps 10
