#!/bin/bash
# Two rocprofv3 PMC passes (8 SQ counters each) + a kernel trace over the FA2 backward kernels at one
# shape; medians per kernel into gpurun_out/fa_bwd_pmc_<tag>.json.   SHAPE="4 16 4096 64 1"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHAPE=${SHAPE:-4 16 4096 64 1}
TAG=${TAG:-d64c}
rm -rf gpurun_out/pmc_$TAG
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc_$TAG/p1 -o run -- python scripts/fa_bwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc_$TAG/p2 -o run -- python scripts/fa_bwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_$TAG/kt -o run -- python scripts/fa_bwd_one.py $SHAPE > /dev/null 2>&1 || exit 1
python - "$TAG" <<'P'
import csv, glob, json, statistics, sys
tag = sys.argv[1]
res = {}


def kind(n):
    for key, name in (("kp", "fa_bwd_kp_kernel"), ("kp_prep", "fa_bwd_kp_prep"), ("kp_dq", "fa_bwd_kp_dq"),
                      ("dq", "fa_bwd_dq"), ("dkdv", "fa_bwd_dkdv"), ("fused", "fa_bwd_fused"),
                      ("hs", "fa_bwd_hs_kernel"), ("hs_prep", "fa_bwd_hs_prep")):
        if name in n:
            return key
    return None

for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    vals = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = kind(n)
        if not k: continue
        vals.setdefault((k, r["Counter_Name"]), {}).setdefault(r["Dispatch_Id"], 0.0)
        vals[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for (k, c), d in vals.items():
        res.setdefault(k, {})[c] = statistics.median(d.values())
for f in glob.glob(f"gpurun_out/pmc_{tag}/kt/**/*kernel_trace.csv", recursive=True):
    ts = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = kind(n)
        if k: ts.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in ts.items():
        res.setdefault(k, {})["duration_us_median"] = statistics.median(v)
for k, d in res.items():
    if d.get("SQ_INSTS_MFMA"):
        d["valu_per_mfma"] = d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"]
    if d.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in d: d[c + "/WAVE_CYCLES"] = d[c] / d["SQ_WAVE_CYCLES"]
json.dump(res, open(f"gpurun_out/fa_bwd_pmc_{tag}.json", "w"), indent=1)
print(json.dumps(res, indent=1))
P
