set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fa_bwd_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
CS336_GEMM_REPORT=gpurun_out/gemm_report_b128.json timeout -k 10 400 python bench.py --batch 128 --steps 10 --warmup 4 > gpurun_out/bench_b128.json 2> gpurun_out/bench_b128.err || { tail -20 gpurun_out/bench_b128.err; exit 1; }
cut -c1-400 gpurun_out/bench_b128.json
timeout -k 10 300 python bench.py --batch 128 --steps 10 --warmup 3 > gpurun_out/bench_b128b.json 2> gpurun_out/bench_b128b.err || { tail -20 gpurun_out/bench_b128b.err; exit 1; }
cut -c1-400 gpurun_out/bench_b128b.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_b96.json 2> gpurun_out/bench_b96.err || { tail -20 gpurun_out/bench_b96.err; exit 1; }
cut -c1-400 gpurun_out/bench_b96.json
grep -o '"peak_mem_gib": [0-9.]*' gpurun_out/bench_b128b.json gpurun_out/bench_b96.json
