#!/bin/bash
# MFMA and LDS busy counters of the gemm8 main loop on its longest-K problem (W1|W3 input gradient,
# 24576 x 1600 x 12800, epilogue ~9 % of the kernel): how close the loop runs to the matrix cores'
# and the LDS array's cycle budgets at the clock the chip actually holds (GRBM_GUI_ACTIVE / 8).
#   bash scripts/pmc_gemm8_mainloop.sh   (on the GPU box; summary in gpurun_out/pmc_g8/summary.txt)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_g8
P="timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_g8/a -o run -- python3 scripts/gemm8w_one.py --nt > gpurun_out/pmc_g8/a.log 2>&1
rc=$?
for f in $(find gpurun_out/pmc_g8 -name '*counter_collection.csv'); do python3 - "$f" <<'PY' | tee gpurun_out/pmc_g8/summary.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if 'gemm8' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in agg.items()}
for k, v in sorted(m.items()):
    print(f"{k} {v:.4g} (mean of {len(agg[k])} calls)")
cyc = m.get('GRBM_GUI_ACTIVE', 0) / 8  # per-XCD kernel cycles
if cyc:
    print(f"kernel cycles (GRBM_GUI_ACTIVE / 8): {cyc:.4g}")
    print(f"MFMA busy / (cycles x 1024 SIMDs): {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024):.3f}")
    print(f"LDS array active / (cycles x 256 CUs): {m.get('SQ_LDS_IDX_ACTIVE', 0) / (cyc * 256):.3f}")
    print(f"LDS bank-conflict share of LDS active: {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}")
PY
done
exit $rc
