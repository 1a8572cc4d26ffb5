"""Workloads ("modes") of the benchmark — the reference's ``benchmark_*`` functions.

``MODES`` maps every mode name of every reference script to its runner:
  * matmul_scaling_benchmark.py: independent | batch_parallel | matrix_parallel
  * backup/matmul_distributed_benchmark.py: independent | data_parallel | model_parallel
  * backup/matmul_overlap_benchmark.py: no_overlap | overlap | pipeline
"""
from __future__ import annotations

from functools import partial

from . import batch_parallel, data_parallel, independent, matrix_parallel, model_parallel, overlap
from .common import ModeResult, Workload

MODES = {
    "independent": independent.run,
    "batch_parallel": batch_parallel.run,
    "matrix_parallel": matrix_parallel.run,
    "data_parallel": data_parallel.run,
    "model_parallel": model_parallel.run,
    "no_overlap": partial(overlap.run, mode="no_overlap"),
    "overlap": partial(overlap.run, mode="overlap"),
    "pipeline": partial(overlap.run, mode="pipeline"),
}

SCALING_MODES = ("independent", "batch_parallel", "matrix_parallel")
DISTRIBUTED_MODES = ("independent", "data_parallel", "model_parallel")
OVERLAP_MODES = ("no_overlap", "overlap", "pipeline")


def run_mode(name: str, w: Workload, ctx) -> ModeResult:
    try:
        fn = MODES[name]
    except KeyError:
        raise ValueError(f"unknown mode {name!r}; choose from {sorted(MODES)}") from None
    return fn(w, ctx)


__all__ = ["MODES", "SCALING_MODES", "DISTRIBUTED_MODES", "OVERLAP_MODES", "ModeResult",
           "Workload", "run_mode"]
