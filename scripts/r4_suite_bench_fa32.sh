#!/bin/bash
# Round-4 check call: full GPU suite (stop after 5 failures), XL bench, and a kernel trace of the fp32
# d128 backward at B 1 H 1 (profiles/r4_flash_sweep.md: the rows slower than materializing PyTorch).
# A GPU fault / abort / timeout (any status other than 0 = pass, 1 = test failures) ends the script.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/r4/suite_full.log 2>&1
rc=$?
tail -15 gpurun_out/r4/suite_full.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_xl.json 2> gpurun_out/r4/bench_xl.err || { tail -20 gpurun_out/r4/bench_xl.err; exit 1; }
cat gpurun_out/r4/bench_xl.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FA_AB_SHAPES="1,1,4096,128,0;1,1,8192,128,0;1,1,16384,128,0;1,1,8192,128,1" FA_AB_DTYPE=fp32 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/fa32 -o run -- python3 scripts/fa_ab.py > gpurun_out/r4/fa32.log 2>&1 || { tail -20 gpurun_out/r4/fa32.log; exit 1; }
grep '^{' gpurun_out/r4/fa32.log
exit $rc
