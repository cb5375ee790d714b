cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
P="timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc/w_sq -o run -- python3 scripts/gemm8w_one.py > gpurun_out/pmc/w_sq.log 2>&1 && \
$P --pmc FETCH_SIZE -d gpurun_out/pmc/w_fetch -o run -- python3 scripts/gemm8w_one.py > gpurun_out/pmc/w_fetch.log 2>&1 && \
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc/nt_sq -o run -- python3 scripts/gemm8w_one.py --nt > gpurun_out/pmc/nt_sq.log 2>&1 && \
$P --pmc FETCH_SIZE -d gpurun_out/pmc/nt_fetch -o run -- python3 scripts/gemm8w_one.py --nt > gpurun_out/pmc/nt_fetch.log 2>&1
rc=$?
for f in $(find gpurun_out/pmc -name '*counter_collection.csv'); do echo "== $f"; python3 - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(list)
for r in rows:
    if 'gemm8' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in agg.items(): print(k, len(v), sum(v)/len(v))
PY
done
exit $rc
