"""Multi-GPU runtime environment, applied before torch (and with it hipBLASLt and RCCL) is loaded.

Why (``profiles/r2_streamk_hang.md``, ``profiles/r3_coresidency.md``): hipBLASLt's picks for the
projection GEMMs on gfx950 are stream-K kernels whose grid is sized to be fully co-resident (<= 1
workgroup per CU, 124 KB LDS each) and whose workgroups spin on flags set by later workgroups of
the same grid. An RCCL collective, in turn, finishes only when all of its channel blocks run. In a
DDP step the bucket all-reduce (RCCL stream) overlaps the backward GEMMs (compute stream); if the
GEMM grid holds every CU, an RCCL kernel can be only partially resident: its missing channel blocks
wait for CUs held by GEMM workgroups, which wait for undispatched successors, which wait for CUs held
by the resident RCCL blocks -- a cycle that crosses ranks through the peers' RCCL kernels.

The cut, as of round 4: the XL bench step has no stream-K kernel left. Every projection GEMM of it,
the vocabulary head included (gemm8 N / K tails), is a cs336 kernel whose workgroups never wait for
other workgroups (committed GEMM table; `profiles/r4_xl_roofline_b96.md` lists no Tensile kernel),
and bench.py's multi-rank DDP-variant sweep runs with ``CS336_GEMM=hip`` for the same reason. What
remains is a cap on stream-K grids (``TENSILE_STREAMK_MAX_CUS``) for any hipBLASLt GEMM that still
runs in a multi-rank job (a shape outside the table takes hipBLASLt's default untimed): it keeps a
reserve of CUs free of stream-K workgroups, where RCCL channel blocks (256 threads, 21 KB LDS, <= 128
VGPRs: several per CU) can always become resident. It costs the bench nothing (no hipBLASLt GEMM runs
in its step). Kernel traces show it does not bind on the projection shapes either: hipBLASLt sizes
their stream-K grids to 224-240 workgroups by itself, and this image's hipBLASLt leaves them
unchanged even at a cap of 128 -- the variable is inert here and kept for builds that honour it
(``profiles/r4_streamk_cap.md``). The RCCL channel cap of round 3 (``NCCL_MAX_NCHANNELS=32``) is dropped: it only bought
safety beside stream-K grids, which the step no longer has, and it capped the all-reduce bandwidth of
every collective. ``scripts/coresidency_probe.py`` / ``tests/test_coresidency_gpu.py`` measure the
stream-K side with an RCCL-shaped cohort (``profiles/r3_coresidency.md``: no stranded cohort in any
configuration, with or without the cap).

Values already in the environment win (``setdefault``), so a user can re-tune either knob.
"""

from __future__ import annotations

import os

N_CU_MI355X = 256
# CUs kept free of stream-K workgroups (an RCCL gfx950 channel block is 256 threads, 21 KB LDS,
# <= 128 VGPRs, so several fit on one free CU)
STREAMK_RESERVE_CUS = 8


def multi_gpu_env(world_size: int, n_cu: int = N_CU_MI355X) -> dict[str, str]:
    """The variables :func:`apply_multi_gpu_env` would set for a ``world_size``-rank job."""
    if world_size <= 1:
        return {}
    return {"TENSILE_STREAMK_MAX_CUS": str(n_cu - STREAMK_RESERVE_CUS)}


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
