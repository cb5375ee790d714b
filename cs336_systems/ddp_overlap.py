"""Reference-path module (``cs336_systems/ddp_overlap.py``): ``DDPOverlap``, the reference's first
attempt at hook-driven overlapped all-reduce. That prototype never constructs (its methods are
nested inside ``__init__``, ``ddp_overlap.py:30-48``) and hard-codes ``/2``; here
the name maps to the working per-parameter overlapped DDP (``DDPIndividual``: async all-reduce from
post-accumulate-grad hooks, mean over the actual world size)."""

from .parallel.ddp import DDPIndividual

DDPOverlap = DDPIndividual

__all__ = ["DDPOverlap"]
