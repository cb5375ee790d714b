from .graphs import GraphedStep
from .memory import allocated_mib, peak_mib, record_memory_history, reset_peak
from .profiling import annotate, annotated, annotations_enabled, enable_annotations
from .timing import StepTimer, do_bench, sync

__all__ = [
    "GraphedStep",
    "allocated_mib",
    "peak_mib",
    "record_memory_history",
    "reset_peak",
    "annotate",
    "annotated",
    "annotations_enabled",
    "enable_annotations",
    "StepTimer",
    "do_bench",
    "sync",
]
