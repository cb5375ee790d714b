#!/bin/bash
# gemm8w (W1|W3 weight gradient, 12800 x 1600 over T tokens) vs gemm8 NT (the equal-FLOP W1|W3 input
# gradient, T x 1600 x 12800): two PMC passes each plus a kernel trace, summarized per counter.
#   bash scripts/pmc_dw_vs_dx.sh [tokens]   (GPU box; gpurun_out/pmc_dwdx/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-52224}; O=gpurun_out/pmc_dwdx; mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for arm in dw dx; do
  flag=""; [ $arm = dx ] && flag="--nt"
  $P --pmc $C1 -d $O/$arm/p1 -o run -- python3 scripts/gemm8w_one.py $flag --tokens $T > $O/${arm}_p1.log 2>&1 || exit $?
  $P --pmc $C2 -d $O/$arm/p2 -o run -- python3 scripts/gemm8w_one.py $flag --tokens $T > $O/${arm}_p2.log 2>&1 || exit $?
  $P -d $O/$arm/kt -o run -- python3 scripts/gemm8w_one.py $flag --tokens $T > $O/${arm}_kt.log 2>&1 || exit $?
  echo "== $arm"; python3 scripts/pmc_summary.py $O/$arm gemm8
done
