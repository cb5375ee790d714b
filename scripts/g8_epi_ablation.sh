#!/bin/bash
# gemm8 SwiGLU epilogue ablation (EPI 1 / EPI 2 at 49152 tokens): the base build against builds that
# drop the epilogue's math, its a/b loads, its stores, or all three (variant libraries built with
# CS336_BUILD_VARIANT="<name> -DCS336_G8_ABL_..."), then one PMC pass over the base EPI 2 kernel.
#   bash scripts/g8_epi_ablation.sh   (GPU box; logs in gpurun_out/g8abl/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/g8abl; mkdir -p $O
for v in base nomath noload nostore bare; do
  lib=cs336_systems/_native/libcs336_hip.so
  [ $v != base ] && lib=cs336_systems/_native/variants/$v/libcs336_hip.so
  CS336_LIB=$lib timeout -k 10 120 python -u scripts/gemm8_stagger.py --settings 0:1 --only swiglu --rounds 3 --no-check \
    > $O/$v.log 2>&1 || exit $?
  echo "$v: $(grep -o '"problem": "[^"]*".*"ms": [0-9.]*' $O/$v.log | sed 's/, "M".*"ms"/ ms/' | tr '\n' ' ')"
done
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d $O/pmc/p1 -o run -- python3 scripts/gemm8_stagger.py --settings 0:1 --only "w2 dX" --rounds 1 --reps 3 > $O/pmc.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv \
  -d $O/pmc/kt -o run -- python3 scripts/gemm8_stagger.py --settings 0:1 --only "w2 dX" --rounds 1 --reps 3 > $O/kt.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/pmc gemm8 > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
