import os, time, json, torch
from cs336_systems.ops._ext import ops as hip_ops
hip = hip_ops()
for N, D in ((256, 32), (8192, 32)):
    q, k, v, do = (torch.randn(1, 1, N, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    o, lse = hip.fa_fwd(q, k, v, True, D**-0.5)
    row = {"N": N}
    for mode in ("split", "nosplit"):
        if mode == "nosplit": os.environ["CS336_FA_BWD_SPLITS"] = "1"
        else: os.environ.pop("CS336_FA_BWD_SPLITS", None)
        for _ in range(20): hip.fa_bwd(do, q, k, v, o, lse, True, D**-0.5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200): hip.fa_bwd(do, q, k, v, o, lse, True, D**-0.5)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        row[mode + "_host_us"] = round((t1 - t0) / 200 * 1e6, 1)
        row[mode + "_total_us"] = round((t2 - t0) / 200 * 1e6, 1)
    print(json.dumps(row), flush=True)
