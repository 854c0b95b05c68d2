"""Offline batch-size profiler (the fork's ModelProfiler, 293-project/profiling/)."""
from .model_profiler import ModelProfiler, ResultsFormatter  # noqa: F401
