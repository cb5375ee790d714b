#!/bin/bash
# kernel traces of hipBLASLt's default GEMM picks with and without the stream-K grid cap
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -rf gpurun_out/sk_cap gpurun_out/sk_nocap
TENSILE_STREAMK_MAX_CUS=248 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sk_cap -o run -- python scripts/streamk_cap_trace.py > gpurun_out/sk_cap.log 2>&1 || { tail gpurun_out/sk_cap.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sk_nocap -o run -- python scripts/streamk_cap_trace.py > gpurun_out/sk_nocap.log 2>&1 || { tail gpurun_out/sk_nocap.log; exit 1; }
python scripts/streamk_cap_trace.py --summarize gpurun_out/sk_cap gpurun_out/sk_nocap | tee gpurun_out/sk_summary.txt
# the knob itself: a cap below the grids hipBLASLt picks must shrink them
if [ "${SK_LOW:-0}" = 1 ]; then
  rm -rf gpurun_out/sk_cap128
  TENSILE_STREAMK_MAX_CUS=128 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sk_cap128 -o run -- python scripts/streamk_cap_trace.py > gpurun_out/sk_cap128.log 2>&1 || { tail gpurun_out/sk_cap128.log; exit 1; }
  python scripts/streamk_cap_trace.py --summarize gpurun_out/sk_cap128 | tee -a gpurun_out/sk_summary.txt
fi
