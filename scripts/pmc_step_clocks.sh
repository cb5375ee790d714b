#!/bin/bash
# Effective clock and MFMA occupancy of every kernel role in one XL training step (real activations,
# not random operands): one rocprofv3 pass with the kernel trace and two counters over bench.py.
#   bash scripts/pmc_step_clocks.sh [bench args...]   (GPU box; gpurun_out/stepclk/, table on stdout)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/stepclk; rm -rf $O; mkdir -p $O
( while sleep 50; do echo "[heartbeat $(date +%T)]"; done ) &
HB=$!; trap "kill $HB" EXIT
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d $O -o run -- python3 bench.py --steps 2 --warmup 1 "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cd scripts && python3 step_clocks.py ../$O
