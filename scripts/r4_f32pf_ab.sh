set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
V=cs336_systems/_native/variants/f32pf/libcs336_hip.so
CS336_LIB=$V timeout -k 10 300 python -u -m pytest -q tests/test_kernels_gpu.py tests/test_flash_long_gpu.py -k "flash" --timeout 120 --timeout-method thread > gpurun_out/r4/f32pf_tests.log 2>&1 || { tail -30 gpurun_out/r4/f32pf_tests.log; exit 1; }
tail -1 gpurun_out/r4/f32pf_tests.log
S="1,1,4096,128,0;1,1,8192,128,0;1,1,16384,128,0;1,1,32768,128,0;1,1,8192,128,1;4,16,4096,128,0;4,16,4096,128,1"
for arm in base f32pf base f32pf; do
  if [ $arm = f32pf ]; then L=$V; else L=; fi
  CS336_LIB=$L FA_AB_SHAPES="$S" FA_AB_DTYPE=fp32 timeout -k 10 200 python -u scripts/fa_ab.py > gpurun_out/r4/f32pf_$arm.log 2>&1 || { tail gpurun_out/r4/f32pf_$arm.log; exit 1; }
  echo "== $arm"; grep '^{' gpurun_out/r4/f32pf_$arm.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['B'],d['H'],d['N'],d['causal'],'fwd',d['fwd_ms'],'bwd',d['bwd_ms'])"
done
