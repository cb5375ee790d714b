cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xlprof${PROF_TAG:-} -o run -- python bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/xlprof${PROF_TAG:-}.log 2>&1 && \
T=$(find gpurun_out/xlprof${PROF_TAG:-} -name '*kernel_trace.csv' | head -n1) && python scripts/roofline_table.py "$T" ${ROOF_ARGS:-} > gpurun_out/xl_roofline${PROF_TAG:-}.md && python scripts/step_sequence.py "$T" ${SEQ_ARGS:-} > gpurun_out/xl_step_sequence${PROF_TAG:-}.txt && \
S=$(find gpurun_out/xlprof${PROF_TAG:-} -name '*kernel_stats.csv' | head -n1) && cp "$S" gpurun_out/xl_kernel_stats${PROF_TAG:-}.csv
