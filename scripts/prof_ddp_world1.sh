#!/bin/bash
# DDP's own cost at world 1: the XL bench step with and without bucketed DDP over a one-rank RCCL
# group (bench.py --ddp-world1), timed (2 interleaved rounds) and then kernel-traced.
#   bash scripts/prof_ddp_world1.sh   (GPU box; gpurun_out/ddpw1/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ddpw1; mkdir -p $O
timeout -k 10 400 python scripts/ab.py bench "plain:" "ddp::--ddp-world1" --rounds 2 --steps 10 || exit $?
for arm in plain ddp; do
  extra=""; [ $arm = ddp ] && extra="--ddp-world1"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$arm -o run -- python3 bench.py --steps 5 --warmup 2 $extra \
    > $O/$arm.log 2>&1 || exit $?
done
python3 scripts/rocpd_diff.py $O/plain/run_results.db $O/ddp/run_results.db 12
