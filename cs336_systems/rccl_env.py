"""Multi-GPU runtime environment, applied before torch (and with it hipBLASLt and RCCL) is loaded.

Why (``profiles/r2_streamk_hang.md``, ``profiles/r3_coresidency.md``): hipBLASLt's picks for the
projection GEMMs on gfx950 are stream-K kernels whose grid is sized to be fully co-resident (<= 1
workgroup per CU, 124 KB LDS each) and whose workgroups spin on flags set by later workgroups of
the same grid. An RCCL collective, in turn, finishes only when all of its channel blocks run. In a
DDP step the bucket all-reduce (RCCL stream) overlaps the backward GEMMs (compute stream); if the
GEMM grid holds every CU, an RCCL kernel can be only partially resident: its missing channel blocks
wait for CUs held by GEMM workgroups, which wait for undispatched successors, which wait for CUs held
by the resident RCCL blocks -- a cycle that crosses ranks through the peers' RCCL kernels.

The cut: cap the stream-K grids (``TENSILE_STREAMK_MAX_CUS``) so that a reserve of CUs never holds a
stream-K workgroup, and cap RCCL's channels (``NCCL_MAX_NCHANNELS``) so that every channel block of a
collective fits on the reserve by itself. Then an RCCL kernel always becomes fully resident (it
needs nothing the GEMM holds), finishes when its peers' do, and the GEMM at worst waits for it.
``scripts/coresidency_probe.py`` / ``tests/test_coresidency_gpu.py`` measure both sides with an
RCCL-shaped cohort that needs all of its workgroups resident at once.

Values already in the environment win (``setdefault``), so a user can re-tune either knob.
"""

from __future__ import annotations

import os

N_CU_MI355X = 256
# CUs kept free of stream-K workgroups, and RCCL channels per collective; an RCCL gfx950 channel
# block is 256 threads, 21 KB LDS, <= 128 VGPRs, so several fit on one free CU
STREAMK_RESERVE_CUS = 8
RCCL_MAX_CHANNELS = 32


def multi_gpu_env(world_size: int, n_cu: int = N_CU_MI355X) -> dict[str, str]:
    """The variables :func:`apply_multi_gpu_env` would set for a ``world_size``-rank job."""
    if world_size <= 1:
        return {}
    return {
        "TENSILE_STREAMK_MAX_CUS": str(n_cu - STREAMK_RESERVE_CUS),
        "NCCL_MAX_NCHANNELS": str(RCCL_MAX_CHANNELS),
    }


def apply_multi_gpu_env(world_size: int | None = None, n_cu: int = N_CU_MI355X) -> dict[str, str]:
    """Set (unless already set) the stream-K / RCCL co-residency caps for a multi-rank run; returns
    what is in effect. Call before ``import torch`` (hipBLASLt and RCCL read these at load/init)."""
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if os.environ.get("CS336_CORESIDENCY_CAP", "1") == "0":
        return {}
    eff = {}
    for k, v in multi_gpu_env(world_size, n_cu).items():
        eff[k] = os.environ.setdefault(k, v)
    return eff
