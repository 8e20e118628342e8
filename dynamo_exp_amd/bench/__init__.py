"""Serving benchmark building blocks shared by bench.py (aggregated, N = 1)
and the disaggregated xPyD body (disagg/bench_disagg.py, N > 1)."""
from .serving import LoadGen, ServingWindow, stagger_lengths  # noqa: F401
