set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py tests/test_fa_rope_gpu.py tests/test_flash_long_gpu.py tests/test_attn_ot_gpu.py tests/test_kernels_gpu.py -k "flash or attn or fa or rope or attention" -m gpu > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -3 gpurun_out/fa_tests.log
for r in 1 2; do
  CS336_LIB=cs336_systems/_native/variants/base/libcs336_hip.so timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_ab_base_$r.jsonl 2>&1 || exit 1
  timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_ab_new_$r.jsonl 2>&1 || exit 1
done
python - <<'P'
import json
for r in (1,2):
  b=[json.loads(l) for l in open(f'gpurun_out/fa_ab_base_{r}.jsonl') if l.startswith('{')]
  n=[json.loads(l) for l in open(f'gpurun_out/fa_ab_new_{r}.jsonl') if l.startswith('{')]
  for x,y in zip(b,n):
    print(r, x['B'],x['H'],x['N'],x['D'],x['causal'],'fwd',x['fwd_tflops'],y['fwd_tflops'],'bwd',x['bwd_tflops'],'->',y['bwd_tflops'])
P
