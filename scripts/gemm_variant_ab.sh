#!/bin/bash
# A/B the cs336 GEMM build variants on one box: default build vs each variants/<name> build.
# usage: scripts/gemm_variant_ab.sh name1 name2 ...
set -u
mkdir -p gpurun_out
timeout -k 10 240 python scripts/gemm_vs_blas.py --json gpurun_out/gemm_ab_default.json > gpurun_out/gemm_ab_default.log 2>&1 || exit $?
for v in "$@"; do
  CS336_LIB=cs336_systems/_native/variants/$v/libcs336_hip.so timeout -k 10 240 python scripts/gemm_vs_blas.py \
    --json gpurun_out/gemm_ab_$v.json > gpurun_out/gemm_ab_$v.log 2>&1 || exit $?
done
python - "$@" <<'PY'
import json, sys
names = ["default"] + sys.argv[1:]
runs = {n: json.load(open(f"gpurun_out/gemm_ab_{n}.json")) for n in names}
for i, r in enumerate(runs["default"]):
    cells = " ".join(f"{n}={runs[n][i].get('cs336_tflops')}" for n in names)
    print(f"{r['shape']:4s} {r['case']:7s} blas={r['blas_tflops']:5d} {cells} err={r.get('max_rel_err')}")
PY
