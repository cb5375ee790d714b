#!/bin/bash
# FA timing: main library vs a variant build (VARIANT=name), both under the same CS336_FA_* env
set -o pipefail
mkdir -p gpurun_out
V=${VARIANT:-dunroll}
CS336_LIB=cs336_systems/_native/variants/$V/libcs336_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py tests/test_flash_long_gpu.py -m gpu > gpurun_out/fa_var_tests.log 2>&1 || { tail -30 gpurun_out/fa_var_tests.log; exit 1; }
tail -1 gpurun_out/fa_var_tests.log
for r in 1 2; do
  timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_var_main_$r.jsonl 2>&1 || exit 1
  CS336_LIB=cs336_systems/_native/variants/$V/libcs336_hip.so timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_var_v_$r.jsonl 2>&1 || exit 1
done
python - <<'P'
import json
for r in (1,2):
  b=[json.loads(l) for l in open(f'gpurun_out/fa_var_main_{r}.jsonl') if l.startswith('{')]
  n=[json.loads(l) for l in open(f'gpurun_out/fa_var_v_{r}.jsonl') if l.startswith('{')]
  for x,y in zip(b,n):
    print(r, x['B'],x['H'],x['N'],x['D'],x['causal'],'fwd',x['fwd_tflops'],y['fwd_tflops'],'bwd',x['bwd_tflops'],'->',y['bwd_tflops'])
P
