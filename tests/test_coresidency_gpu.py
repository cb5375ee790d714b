"""RCCL co-residency beside stream-K GEMMs (VERDICT r2 "next" 1b).

A DDP step overlaps the bucket all-reduce (RCCL stream) with the backward GEMMs (compute stream).
hipBLASLt's stream-K GEMM workgroups wait for later workgroups of their own grid; an RCCL kernel
finishes only when all of its channel blocks run. A partially resident RCCL kernel beside a
partially resident stream-K grid is the cross-rank deadlock to rule out. The probe
(scripts/coresidency_probe.py) launches an RCCL-shaped cohort -- 256 threads, 21 KB LDS, 128 VGPRs
per workgroup, every workgroup waiting until all of them are resident (bounded by a deadline, so a
stranded cohort reports instead of hanging) -- released at the same moment as EACH GEMM of the XL
backward sequence, i.e. racing the GEMM grid for the CUs. Run in a child process because the
stream-K/RCCL caps (cs336_systems/rccl_env.py) must be in the environment before torch loads.
"""

import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _probe(env_extra: dict, blocks: int) -> dict:
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, os.path.join(REPO, "scripts", "coresidency_probe.py"), "--race", "--iters", "10",
           "--deadline-ms", "20", "--blocks", str(blocks)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    print(json.dumps(res))
    return res


def test_cohort_never_stranded_with_multi_gpu_caps():
    from cs336_systems.rccl_env import multi_gpu_env

    env = multi_gpu_env(8)
    res = _probe(env, 64)  # an uncapped RCCL collective's channel blocks beside capped stream-K grids
    assert res["env"].get("TENSILE_STREAMK_MAX_CUS") == env["TENSILE_STREAMK_MAX_CUS"]
    assert res["cohort_timeouts_wg"] == 0, res
    assert res["results_bitwise_equal"]


def test_cohort_beside_uncapped_streamk_gemms():
    """Without the caps (hipBLASLt's default full-chip stream-K grids), 128 RCCL-shaped blocks:
    measured 0 stranded cohorts in every configuration so far (profiles/r3_coresidency.md); kept as
    a tripwire for a hipBLASLt/RCCL update that changes it."""
    res = _probe({"CS336_CORESIDENCY_CAP": "0"}, 128)
    assert res["cohort_timeouts_wg"] == 0, res
    assert res["results_bitwise_equal"]
