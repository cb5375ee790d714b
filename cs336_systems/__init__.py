"""cs336_systems (MI355X-native): Transformer-LM systems stack for AMD Instinct MI355X (gfx950).

Layers: ``models`` (Transformer LM, configs), ``ops`` (HIP/CDNA4 kernels + eager references),
``parallel`` (RCCL data parallel variants, ZeRO-1 sharded optimizer), ``utils`` (timing, memory,
roctx), ``bench`` (benchmark/profiling drivers). Reference-compatible module names
(``flash_attention``, ``ddp_bucketed_overlapped_sharded``, ``benchmark``, ...) re-export these.
"""

__version__ = "0.1.0"
