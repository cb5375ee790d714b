#!/bin/bash
# (1) the 8-wave head-sequential backward (fa_bwd_fused.hip, CS336_FA_BWD=1) against the two-kernel
# form on the only shapes the default selection gives it (B·H >= 512, N <= 1024, N % 128 == 64);
# (2) kernel trace of the B 1 H 1 small-N backward (launch count and time per kernel).
#   bash scripts/fa_small_probe.sh   (GPU box; gpurun_out/fasmall/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/fasmall; mkdir -p $O
export FA_AB_SHAPES="64,16,448,64,1;64,16,448,64,0;96,25,192,64,1;32,32,960,64,1"
timeout -k 10 300 python scripts/ab.py fa "two:CS336_FA_BWD=0" "fused:CS336_FA_BWD=1" "default:" --rounds 2 || exit $?
export FA_AB_SHAPES="1,1,256,32,1;1,1,512,32,1;1,1,1024,64,1;1,1,2048,64,1"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o run -- python3 scripts/fa_ab.py > $O/kt.log 2>&1 || exit $?
grep '^{' $O/kt.log
python3 scripts/rocpd_summary.py $O/kt/run_results.db "fa_|rope|fill|copy|reduce|elementwise" | head -60
