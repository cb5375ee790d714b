#!/bin/bash
# VERDICT r2 #4 evidence: a 2-rank (gloo, one GPU) ZeRO rehearsal under rocprofv3 --kernel-trace;
# counts the transpose kernels per process. With the Wᵀ shadows refreshed after every all-gather
# (sharded_optimizer._after_gather / zero.py) the forward transposes no weight: the only transposes
# left are the ones the fused AdamW does inside its own kernel.
# usage: scripts/zero_transpose_count.sh [--sharded | --ddp zero]  -> gpurun_out/zero_tr_<tag>.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-zero2}
export CS336_DIST_BACKEND=gloo
rm -rf gpurun_out/zero_tr_$TAG
# two ranks started directly (no launcher process under the profiler): each python is its own
# rocprofv3 target
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zero_tr_$TAG/rank$r -o run -- \
    python bench.py --gpus 2 --steps 2 --warmup 1 --batch 8 "$@" > gpurun_out/zero_tr_${TAG}_rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { echo "rank failed rc=$rc"; tail -5 gpurun_out/zero_tr_${TAG}_rank*.log; exit 1; }
python - "$TAG" <<'P' | tee gpurun_out/zero_tr_$TAG.txt
import csv, glob, sys, collections
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/zero_tr_{tag}/**/*kernel_trace.csv", recursive=True)):
    pids = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        key = "transpose" if "transpose" in n.lower() else ("gemm8w" if "gemm8w" in n else ("gemm8" if "gemm8" in n else None))
        pids[f]["kernels"] += 1
        if key:
            pids[f][key] += 1
    for pid, c in pids.items():
        print(pid, dict(c))
P
