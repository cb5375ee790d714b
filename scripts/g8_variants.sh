#!/bin/bash
# Time gemm8's SwiGLU / plain epilogue problems (scripts/gemm8_epi_bench.py, 49152 tokens) under every
# variant library in cs336_systems/_native/variants/ and the base build, interleaved twice.
#   bash scripts/g8_variants.sh [--only swiglu]   (GPU box; logs in gpurun_out/g8var/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/g8var; mkdir -p $O
for r in 1 2; do
  for v in base $(ls cs336_systems/_native/variants); do
    lib=cs336_systems/_native/libcs336_hip.so
    [ $v != base ] && lib=cs336_systems/_native/variants/$v/libcs336_hip.so
    CS336_LIB=$lib timeout -k 10 150 python -u scripts/gemm8_epi_bench.py --rounds 2 --no-check "$@" \
      > $O/${v}_$r.log 2>&1 || exit $?
    echo "r$r $v: $(grep -o '"problem": "[^"]*".*"ms": [0-9.]*' $O/${v}_$r.log | sed 's/"problem": //; s/, "M".*"ms"//' | tr '\n' ' ')"
  done
done
