"""Workloads ("modes") of the benchmark — the reference's ``benchmark_*`` functions.

``MODES`` maps every mode name of every reference script to its runner:
  * matmul_scaling_benchmark.py: independent | batch_parallel | matrix_parallel
    (+ ring_parallel, an MI355X addition: all-gather-GEMM over the xGMI ring)
  * backup/matmul_distributed_benchmark.py: independent | data_parallel | model_parallel
  * backup/matmul_overlap_benchmark.py: no_overlap | overlap | pipeline
"""
from __future__ import annotations

from enum import Enum
from functools import partial

from . import (batch_parallel, data_parallel, independent, matrix_parallel, model_parallel, overlap,
               ring_parallel)
from .common import ModeResult, Workload

MODES = {
    "independent": independent.run,
    "batch_parallel": batch_parallel.run,
    "matrix_parallel": matrix_parallel.run,
    "ring_parallel": ring_parallel.run,
    "data_parallel": data_parallel.run,
    "model_parallel": model_parallel.run,
    "no_overlap": partial(overlap.run, mode="no_overlap"),
    "overlap": partial(overlap.run, mode="overlap"),
    "pipeline": partial(overlap.run, mode="pipeline"),
}

SCALING_MODES = ("independent", "batch_parallel", "matrix_parallel")
# Selectable in matmul_scaling_benchmark.py beyond the reference's three.
EXTRA_SCALING_MODES = ("ring_parallel",)


class ScalingMode(Enum):
    """matmul_scaling_benchmark.py:10-13."""
    INDEPENDENT = "independent"
    BATCH_PARALLEL = "batch_parallel"
    MATRIX_PARALLEL = "matrix_parallel"


class BenchmarkMode(Enum):
    """backup/matmul_distributed_benchmark.py:10-13 and backup/matmul_overlap_benchmark.py:11-14."""
    INDEPENDENT = "independent"
    DATA_PARALLEL = "data_parallel"
    MODEL_PARALLEL = "model_parallel"
    NO_OVERLAP = "no_overlap"
    OVERLAP = "overlap"
    PIPELINE = "pipeline"


DISTRIBUTED_MODES = ("independent", "data_parallel", "model_parallel")
OVERLAP_MODES = ("no_overlap", "overlap", "pipeline")


def run_mode(name, w: Workload, ctx) -> ModeResult:
    if isinstance(name, Enum):
        name = name.value
    try:
        fn = MODES[name]
    except KeyError:
        raise ValueError(f"unknown mode {name!r}; choose from {sorted(MODES)}") from None
    return fn(w, ctx)


__all__ = ["MODES", "SCALING_MODES", "EXTRA_SCALING_MODES", "DISTRIBUTED_MODES", "OVERLAP_MODES", "ModeResult",
           "Workload", "run_mode", "ScalingMode", "BenchmarkMode"]
