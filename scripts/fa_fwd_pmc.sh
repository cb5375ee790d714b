#!/bin/bash
# Two rocprofv3 PMC passes + a kernel trace over the FA2 forward kernel at one shape (SHAPE="B H N D causal").
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHAPE=${SHAPE:-96 25 512 64 1}
TAG=${TAG:-xl}
rm -rf gpurun_out/fpmc_$TAG
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/fpmc_$TAG/p1 -o run -- python scripts/fa_fwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/fpmc_$TAG/p2 -o run -- python scripts/fa_fwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/fpmc_$TAG/p3 -o run -- python scripts/fa_fwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fpmc_$TAG/kt -o run -- python scripts/fa_fwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
echo ok
