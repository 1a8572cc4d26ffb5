"""``batch_parallel`` mode: data-parallel batched GEMM + RCCL all-reduce of the
output (a gradient-sync stand-in).

Reference: matmul_scaling_benchmark.py:106-165. Global batch 4 split
``4 // ws`` per rank, ``bmm`` then ``all_reduce(C, SUM)``; compute and comm
are timed separately with host syncs inside the loop and reported as
TFLOPS = 2N³·local_b / (t_compute + t_comm).

Differences:
  * Q3: the global batch is rounded up to a multiple of ws (≥ 4), so ws=8
    runs one 16k GEMM per rank instead of an empty batch; reported FLOPs are
    the FLOPs actually executed.
  * Q10: segment boundaries are hipEvents recorded on the stream; the host
    never synchronises inside the timed loop.
  * ``overlap=True``: the local batch is cut into units (batch element ×
    row chunk). Unit u's GEMM runs on the compute stream; its all-reduce
    runs on a high-priority comm stream as soon as u's ready-event fires,
    while unit u+1 computes. The next iteration's GEMM into a unit waits for
    that unit's done-event (no write-while-reducing race, Q7). Time per
    iteration is then wall time; compute-only time is measured in a separate
    loop and both are reported (Q9).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel.comm import current_stream
from ..parallel.overlap import ReduceOverlap, compute_ctx, compute_stream, gemm_chunks
from ..parallel.dist import DistContext
from ..parallel.partition import global_batch, local_batch
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import SegmentTimer, Stopwatch, synchronize, time_loop_ms
from .common import (ModeResult, Workload, align_ranks, allreduced_relerr, gemm_fn, kernel_label,
                     out_dtype, randn, warmup)


def run(w: Workload, ctx: DistContext) -> ModeResult:
    dev, n, ws = ctx.device, w.n, ctx.world_size
    gb = global_batch(ws, w.batch)
    lb = local_batch(ws, w.batch)
    A = randn((lb, n, n), w, dev, seed=2 * (w.seed + ctx.rank))
    B = randn((lb, n, n), w, dev, seed=2 * (w.seed + ctx.rank) + 1, operand="B")
    C = torch.empty((lb, n, n), device=dev, dtype=out_dtype(w))
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A, B, C)
    distributed = ctx.is_distributed
    flops = gemm_flops(n, n, n, lb)

    def reduce_all():
        if distributed:
            dist.all_reduce(C)

    extra = {"global_batch": gb, "local_batch": lb, "overlap": bool(w.overlap and distributed)}
    if not (w.overlap and distributed):
        def serial_step():
            mm(A, B, C)
            reduce_all()

        warmup(serial_step, w, ctx)
        align_ranks(ctx)
        seg = SegmentTimer(dev)
        stream = current_stream(dev)
        seg.begin(stream)
        for _ in range(w.iters):
            mm(A, B, C)
            seg.mark("compute", stream)
            reduce_all()
            seg.mark("comm", stream)
        tot = seg.totals_ms()
        it = max(w.iters, 1)
        comp = tot.get("compute", 0.0) / it
        comm = tot.get("comm", 0.0) / it
        avg = comp + comm
        res = ModeResult(mode="batch_parallel", n=n, world_size=ws, avg_ms=avg,
                         flops_local=flops, flops_total=flops * ws,
                         tflops=tflops_from(flops, avg / 1e3), compute_ms=comp, comm_ms=comm,
                         compute_only_tflops=tflops_from(flops, comp / 1e3), kernel=label,
                         extra=extra)
    else:
        ov = ReduceOverlap(lb, gemm_chunks(n, n, w.chunks, w.dtype, dev), dev)
        extra["units"] = len(ov.units)
        _, s0, e0 = ov.units[0]  # what a chunk runs beside the reductions
        label = kernel_label(w, A[0, s0:e0], B[0], C[0, s0:e0], shared=True)
        compute, owner = compute_stream(dev, w.comm_cus)
        extra["comm_cus"] = w.comm_cus

        def step():
            with compute_ctx(compute, owner):
                ov.step(mm, A, B, C, compute)
            if compute is not None:  # the timing stream joins the (masked) compute stream
                current_stream(dev).wait_stream(compute)

        warmup(step, w, ctx)
        # compute-only reference time (reference: 10 GEMM-only iterations), taken
        # BEFORE the timed loop so the loop's last reduced C stays checkable.
        synchronize(dev)
        k = max(1, min(w.iters, 10))
        comp = time_loop_ms(lambda: mm(A, B, C), k, 0, dev) / k
        align_ranks(ctx)
        sw = Stopwatch(dev)
        sw.start(current_stream(dev))
        for _ in range(w.iters):
            step()
        sw.stop(current_stream(dev))
        avg = sw.elapsed_ms() / max(w.iters, 1)
        res = ModeResult(mode="batch_parallel", n=n, world_size=ws, avg_ms=avg,
                         flops_local=flops, flops_total=flops * ws,
                         tflops=tflops_from(flops, avg / 1e3), compute_ms=comp,
                         comm_ms=max(avg - comp, 0.0),
                         compute_only_tflops=tflops_from(flops, comp / 1e3), kernel=label,
                         extra=extra)
    if w.check:
        # Every timed iteration recomputes C and all-reduces it, so after the
        # loop C[b] must equal Σ_ranks A_r[b] @ B_r[b] (checks GEMM + RCCL +
        # the overlap event ordering end to end).
        synchronize(dev)
        res.relerr = max(allreduced_relerr(ctx, A[b], B[b], C[b]) for b in range(lb))
    return res
