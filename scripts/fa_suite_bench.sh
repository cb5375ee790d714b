set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py tests/test_fa_rope_gpu.py tests/test_flash_long_gpu.py tests/test_attn_ot_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
timeout -k 10 300 python -m cs336_systems.bench.flash --impls hip_fa2 torch_sdpa --no-compile --json gpurun_out/flash4096.json > gpurun_out/flash4096.log 2>&1 || { tail gpurun_out/flash4096.log; exit 1; }
timeout -k 10 300 python -m cs336_systems.bench.flash --leaderboard --impls hip_fa2 --no-compile --json gpurun_out/flash_leaderboard.json > gpurun_out/flash_lb.log 2>&1 || { tail gpurun_out/flash_lb.log; exit 1; }
python - <<'P'
import json
for f in ('gpurun_out/flash4096.json','gpurun_out/flash_leaderboard.json'):
  for r in json.load(open(f)):
    print(r.get('impl'), r.get('B'), r.get('H'), r.get('N'), r.get('d'), r.get('causal'), 'fwd', round(r.get('fwd_tflops',0)), 'bwd', round(r.get('bwd_tflops',0)), 'fwd+bwd ms', round(r.get('fwd_bwd_ms',0),3))
P
timeout -k 10 300 python bench.py --model 2.7b --ctx 1024 --batch 12 --steps 10 --warmup 3 > gpurun_out/bench_2p7b.json 2> gpurun_out/bench_2p7b.err || { tail -20 gpurun_out/bench_2p7b.err; exit 1; }
cat gpurun_out/bench_2p7b.json
