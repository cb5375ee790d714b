#!/bin/bash
# One gpurun call, staged checks; replaces final_check.sh / session_end_check.sh /
# gpu_suite_bench_prof.sh / fa_suite_bench.sh. Each GPU step runs under its own time limit and the
# chain stops at the first failure (nothing else touches a sick GPU).
#   bash scripts/gpu_check.sh suite bench 2p7b prof flash leaderboard rehearse
# stages: suite (pytest -m gpu), bench (XL default, 20 steps), 2p7b (2.7b ctx 1024 batch 12),
#         prof (rocprofv3 kernel trace of the XL step -> roofline + step sequence; PROF_TAG names it),
#         flash (FA2 at N 4096, d 64/128), leaderboard ((16,16384,64) causal fwd+bwd, cold caches),
#         rehearse (2 ranks on one GPU over gloo through bench.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for stage in "$@"; do
  case $stage in
    suite)
      timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -40 gpurun_out/gpu_suite.log; exit 1; }
      tail -1 gpurun_out/gpu_suite.log ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_xl.json 2> gpurun_out/bench_xl.err || { tail -20 gpurun_out/bench_xl.err; exit 1; }
      cat gpurun_out/bench_xl.json ;;
    2p7b)
      timeout -k 10 300 python bench.py --model 2.7b --ctx 1024 --batch 12 --steps 10 --warmup 3 > gpurun_out/bench_2p7b.json 2> gpurun_out/bench_2p7b.err || { tail -20 gpurun_out/bench_2p7b.err; exit 1; }
      cut -c1-220 gpurun_out/bench_2p7b.json ;;
    prof)
      bash scripts/prof_xl_step.sh || exit 1
      head -16 gpurun_out/xl_roofline${PROF_TAG:-}.md ;;
    flash)
      timeout -k 10 300 python -m cs336_systems.bench.flash --impls hip_fa2 --no-compile --json gpurun_out/flash4096.json > gpurun_out/flash4096.log 2>&1 || { tail gpurun_out/flash4096.log; exit 1; }
      python -c "
import json
for r in json.load(open('gpurun_out/flash4096.json')):
    print(r['impl'], r['N'], r['d'], r['causal'], 'fwd', round(r['fwd_tflops']), 'bwd', round(r['bwd_tflops']))" ;;
    leaderboard)
      timeout -k 10 300 python -m cs336_systems.bench.flash --leaderboard --impls hip_fa2 --json gpurun_out/flash_leaderboard.json > gpurun_out/flash_lb.log 2>&1 || { tail gpurun_out/flash_lb.log; exit 1; }
      cat gpurun_out/flash_leaderboard.json ;;
    rehearse)
      timeout -k 10 300 bash scripts/rehearse_multirank.sh > gpurun_out/rehearse.log 2>&1 || { tail -30 gpurun_out/rehearse.log; exit 1; }
      grep '"metric"' gpurun_out/rehearse.log | cut -c1-300 ;;
    quick)  # QUICK_TESTS="tests/a.py tests/b.py": a targeted subset of the GPU suite
      timeout -k 10 600 python -u -m pytest ${QUICK_TESTS:-tests/test_train_graph_gpu.py} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_quick.log 2>&1 || { tail -60 gpurun_out/gpu_quick.log; exit 1; }
      tail -3 gpurun_out/gpu_quick.log ;;
    stamps)  # in-kernel gemm8 phase stamps (CS336_G8_STAMP variant build)
      CS336_LIB=cs336_systems/_native/variants/stamp/libcs336_hip.so timeout -k 10 300 python -u scripts/gemm8_stamps.py ${STAMP_ARGS:-} --json gpurun_out/gemm8_stamps.json > gpurun_out/gemm8_stamps.log 2>&1 || { tail -30 gpurun_out/gemm8_stamps.log; exit 1; }
      cat gpurun_out/gemm8_stamps.log ;;
    graphab)  # eager step vs the whole step captured in one HIP graph, same box
      timeout -k 10 900 python scripts/ab.py bench "eager:" "graphs:PYTHONFAULTHANDLER=1:--graphs on" --rounds ${AB_ROUNDS:-2} --steps 10 --timeout 300 > gpurun_out/graphab.log 2>&1 || { tail -30 gpurun_out/graphab.log; exit 1; }
      tail -8 gpurun_out/graphab.log ;;
    dwab)  # weight-gradient GEMMs as the step runs them: base variant lib vs this tree's lib, interleaved
      for r in 1 2; do
        for v in base new; do
          lib=cs336_systems/_native/libcs336_hip.so; [ $v = base ] && lib=cs336_systems/_native/variants/base/libcs336_hip.so
          CS336_LIB=$lib timeout -k 10 240 python -u scripts/dw_time.py --tag "$v$r" >> gpurun_out/dwab.log 2>&1 || { tail -20 gpurun_out/dwab.log; exit 1; }
        done
      done
      grep '^{' gpurun_out/dwab.log ;;
    ddpw1)  # DDP's own cost at world 1 (no collectives since round 6): plain step vs the bucketed wrapper
      timeout -k 10 1200 python scripts/ab.py bench "plain::--overlap-opt off" "ddpw1::--ddp-world1" "ddpw1ov::--ddp-world1 --overlap-opt on" --rounds ${AB_ROUNDS:-2} --steps 10 --timeout 300 > gpurun_out/ddpw1.log 2>&1 || { tail -30 gpurun_out/ddpw1.log; exit 1; }
      cat gpurun_out/ddpw1.log ;;
    emul)  # emulated W = 8 communication beside the real XL backward (byte-moving occupants)
      timeout -k 10 900 python -u scripts/comm_emulation.py ${EMUL_ARGS:-} > gpurun_out/comm_emulation.jsonl 2> gpurun_out/comm_emulation.err || { tail -30 gpurun_out/comm_emulation.err; exit 1; }
      cat gpurun_out/comm_emulation.jsonl ;;
    numa)  # 1-GPU bench with / without the host pinned to the GPU's NUMA-local CPUs
      timeout -k 10 1200 python scripts/ab.py bench "pin:" "nopin:CS336_NUMA_PIN=0" "pin_ovoff::--overlap-opt off" --rounds ${AB_ROUNDS:-2} --steps 10 --timeout 300 > gpurun_out/numa.log 2>&1 || { tail -30 gpurun_out/numa.log; exit 1; }
      cat gpurun_out/numa.log ;;
    cveprof)  # kernel traces of the eager and the compiled e2e step (CVE_SIZE, batch 4, ctx 512)
      cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
      for m in eager compile; do
        flag=""; [ $m = compile ] && flag="--compile"
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cve_$m -o run -- python -u -m cs336_systems.bench.e2e --sizes ${CVE_SIZE:-2.7b} --ctx 512 --mixed $flag --json gpurun_out/cve_$m.json > gpurun_out/cve_$m.log 2>&1 || { tail -20 gpurun_out/cve_$m.log; exit 1; }
        cp $(find gpurun_out/cve_$m -name '*kernel_stats.csv' | head -n1) gpurun_out/cve_${m}_kernel_stats.csv
        cat gpurun_out/cve_$m.json
      done ;;
    faab)  # FA2 arms (FA_ARMS: ab.py arm specs, ';'-separated) over shapes (FA_SHAPES: bench.flash arg sets, ';'-separated)
      IFS=';' read -ra arms <<< "${FA_ARMS:-default:}"
      IFS=';' read -ra shapes <<< "${FA_SHAPES:---seq 1024 --batch 32 --heads 32 --d 80 --causal 1}"
      for sh in "${shapes[@]}"; do
        timeout -k 10 900 python scripts/ab.py flash "${arms[@]}" --args "$sh" --rounds 2 --timeout 240 > gpurun_out/faab.log 2>&1 || { tail -30 gpurun_out/faab.log; exit 1; }
        grep '^round' gpurun_out/faab.log | sed 's/hip_fa2 //' | cut -c1-150 | tee -a gpurun_out/faab_all.log
      done ;;
    benchab)  # bench.py arms (BENCH_ARMS, ';'-separated) with BENCH_ARGS for every arm
      IFS=';' read -ra arms <<< "${BENCH_ARMS:-default:}"
      timeout -k 10 1200 python scripts/ab.py bench "${arms[@]}" --args "${BENCH_ARGS:-}" --rounds ${AB_ROUNDS:-2} --steps 10 --timeout 300 > gpurun_out/benchab.log 2>&1 || { tail -30 gpurun_out/benchab.log; exit 1; }
      grep '^round' gpurun_out/benchab.log ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
