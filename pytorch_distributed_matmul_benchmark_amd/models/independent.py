"""``independent`` mode: every rank runs its own full N×N GEMM; no collectives.

Reference: matmul_benchmark.py:39-79 (``benchmark_matmul``) and
matmul_scaling_benchmark.py:69-104 (``benchmark_independent``): per-rank seed,
A,B = randn(N,N), warmup, sync + barrier, one event pair around ``iters``
back-to-back GEMMs. This is the perfect-scaling ceiling of the node.

Here the timed loop is native on GPU: ``ops.gemm.bench_matmul`` records two
hipEvents around ``iters`` launches of the MFMA kernel issued from C++ (no
Python, no allocator in the loop), optionally replayed as one hipGraph.
TFLOPS = 2N³ / t per rank; the node figure is the SUM over ranks.
"""
from __future__ import annotations

import torch

from ..ops import gemm as _gemm
from ..parallel.dist import DistContext
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import time_loop_ms
from .common import (ModeResult, Workload, align_ranks, gemm_fn, kernel_label, out_dtype, randn,
                     sampled_relerr, warmup)


def run(w: Workload, ctx: DistContext, mode_name: str = "independent") -> ModeResult:
    dev = ctx.device
    n = w.n
    A = randn((n, n), w, dev, seed=2 * (w.seed + ctx.rank))
    B = randn((n, n), w, dev, seed=2 * (w.seed + ctx.rank) + 1, operand="B")
    C = torch.empty((n, n), device=dev, dtype=out_dtype(w))
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A, B, C)

    warmup(lambda: mm(A, B, C), w, ctx)
    align_ranks(ctx)
    if dev.type == "cuda" and w.backend == "native":
        total_ms = _gemm.bench_matmul(A, B, C, w.iters, 0, graph=w.graph, kernel=w.kernel)
    else:
        total_ms = time_loop_ms(lambda: mm(A, B, C), w.iters, 0, dev)
    avg_ms = total_ms / max(w.iters, 1)
    flops = gemm_flops(n, n, n)
    res = ModeResult(mode=mode_name, n=n, world_size=ctx.world_size, avg_ms=avg_ms,
                     flops_local=flops, flops_total=flops * ctx.world_size,
                     tflops=tflops_from(flops, avg_ms / 1e3), compute_ms=avg_ms, comm_ms=0.0,
                     kernel=label)
    if w.check:
        res.relerr = sampled_relerr(A, B, C)
    return res
