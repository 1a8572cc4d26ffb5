"""backup ``model_parallel`` mode, fixed.

Reference: backup/matmul_distributed_benchmark.py:112-174 intends a column
split but multiplies ``A[:, s:e] @ B_local`` = [N, N/ws] @ [N, N/ws], a shape
error for every ws > 1, so it never produced a number. Here it
is the column-parallel GEMM of ``matrix_parallel`` (replicated A, B column
shard, all-gather of the C blocks) reported the backup way: TFLOPS =
2N³ / t_total (whole-op rate), plus compute / comm / overhead.
"""
from __future__ import annotations

from ..parallel.dist import DistContext
from ..utils.metrics import tflops_from
from . import matrix_parallel
from .common import ModeResult, Workload


def run(w: Workload, ctx: DistContext) -> ModeResult:
    r = matrix_parallel.run(w, ctx)
    r.mode = "model_parallel"
    r.tflops = tflops_from(r.flops_total, r.avg_ms / 1e3)
    return r
