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
  * ``overlap=True`` (parallel/overlap.py OverlapPipeline): each batch
    element is one whole GEMM (a unit); its all-reduce runs on a
    high-priority comm stream while the next element — or the next
    iteration's first — computes, and the next GEMM into a buffer waits
    only for that buffer's last all-reduce (no write-while-reducing race,
    Q7). With one element per rank (ws >= 4) the ring has a second C, the
    reference's C1/C2 (backup/matmul_overlap_benchmark.py:98-101). Where the
    planner says so, the all-reduce of an element starts piece by piece as
    the GEMM's own tiles complete (W4 completion signals). A plan that loses
    to serializing runs serialized. Time per iteration is wall time; the
    compute-only time is measured in a separate loop, under the same
    shared-device context the pipeline's GEMMs run in, and both are reported
    (Q9).
"""
from __future__ import annotations

import torch
from ..parallel.comm import CommStream, current_stream
from ..parallel.ipc import ipc_empty
from ..parallel.overlap import (OverlapPipeline, all_reduce_now, compute_ctx, compute_stream,
                                ipc_buffers, make_gatherer, measured_plan, pick_collective,
                                reduce_fn)
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
    # --allreduce ipc / auto: peers may pull chunks straight out of C (IPC-exportable allocations)
    alloc = ((lambda *shape: ipc_empty(shape, out_dtype(w), dev)) if ipc_buffers(w.allreduce, dev)
             else (lambda *shape: torch.empty(shape, device=dev, dtype=out_dtype(w))))
    C = alloc(lb, n, n)
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A, B, C)
    distributed = ctx.is_distributed
    flops = gemm_flops(n, n, n, lb)

    def reduce_all():  # `impl` / `direct` (the collective and its comm object) are bound below
        if distributed:
            all_reduce_now(C, impl, direct)

    extra = {"global_batch": gb, "local_batch": lb, "overlap": bool(w.overlap and distributed),
             "allreduce": w.allreduce}
    plan = None
    units = ([(A[b], B[b], C[b]) for b in range(lb)] if lb >= 2 else
             [(A[0], B[0], C[0]), (A[0], B[0], alloc(n, n))])
    cs = CommStream(dev)
    # the collective's comm object: the CommStream, or (--allreduce ipc on GPUs)
    # an IpcGather with every output buffer registered; auto: the fastest of
    # rccl / direct / ipc on this job's ranks (pick_collective)
    srcs = [C] + ([units[1][2]] if lb == 1 else [])
    impl = w.allreduce
    if impl == "auto" and distributed:
        spread = {}
        impl, direct, times = pick_collective(ctx, "all_reduce", units[0][2], srcs, comm=cs,
                                              spread_out=spread)
        extra["allreduce"], extra["collective_us"] = f"auto:{impl}", times
        extra["collective_spread_us"] = spread
    else:
        impl = "rccl" if impl == "auto" else impl
        direct = make_gatherer(impl, dev, srcs, comm=cs) if impl != "rccl" and distributed else None
    compute, owner = (compute_stream(dev, w.comm_cus) if (w.overlap and distributed)
                      else (current_stream(dev), None))
    ar = reduce_fn(impl, direct if direct is not None else cs)
    if w.overlap and distributed:
        # priced from this job's own GEMM and all-reduce times (MAX over ranks)
        plan = measured_plan(units, ctx, "all_reduce", n * n * C.element_size(), mm,
                             lambda s, e: ar(units[0][2][s:e]), native=w.backend == "native",
                             requested=w.chunks, steps=max(w.iters, 1), compute=compute,
                             owner=owner, comm=cs)
        extra["plan"] = plan.as_dict()
    if plan is None or not plan.overlap:
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
        checked = [(b, C[b]) for b in range(lb)]
    else:
        def coll(r, p, s, e, after, done):
            ar(units[r][2][s:e], after=after, done=done)

        pipe = OverlapPipeline(mm, units, coll, dev, plan, per_step=lb, compute=compute,
                               owner=owner, comm=cs)
        extra["units_per_step"] = lb
        extra["ring"] = len(units)
        extra["pieces"] = len(pipe.pieces)
        extra["signalled"] = pipe.signalled
        extra["comm_cus"] = len(owner.excluded) if owner is not None else 0
        label = ("pdmb_w4_nn (completion signals)" if pipe.signalled
                 else kernel_label(w, A[0], B[0], C[0], shared=True))

        def step():
            pipe.step()

        def finish():
            pipe.finish()
            if compute is not None:  # the timing stream joins the (masked) compute stream
                current_stream(dev).wait_stream(compute)

        warmup(lambda: (step(), finish()), w, ctx)
        # compute-only reference time (reference: 10 GEMM-only iterations) of the
        # same GEMMs in the same context (shared device / CU budget), taken BEFORE
        # the timed loop so the loop's last reduced C stays checkable.
        synchronize(dev)
        k = max(1, min(w.iters, 10))

        scratch = torch.empty_like(C[0])  # the ring's outputs keep their reduced values

        def gemms_only():
            with compute_ctx(compute, owner):
                for b in range(lb):
                    mm(A[b], B[b], scratch)
            if compute is not None:
                current_stream(dev).wait_stream(compute)
        comp = time_loop_ms(gemms_only, k, 0, dev) / k
        align_ranks(ctx)
        sw = Stopwatch(dev)
        sw.start(current_stream(dev))
        for _ in range(w.iters):
            step()
        finish()
        sw.stop(current_stream(dev))
        avg = sw.elapsed_ms() / max(w.iters, 1)
        pipe.close()
        res = ModeResult(mode="batch_parallel", n=n, world_size=ws, avg_ms=avg,
                         flops_local=flops, flops_total=flops * ws,
                         tflops=tflops_from(flops, avg / 1e3), compute_ms=comp,
                         comm_ms=max(avg - comp, 0.0),
                         compute_only_tflops=tflops_from(flops, comp / 1e3), kernel=label,
                         extra=extra)
        # only the ring slots the pipeline wrote (a slot never used holds no sum)
        checked = [(i, u[2]) for i, (u, used) in enumerate(zip(units, pipe.used)) if used]
    if w.check:
        # Every timed iteration recomputes C and all-reduces it, so after the
        # loop C[b] must equal Σ_ranks A_r[b] @ B_r[b] (checks GEMM + RCCL +
        # the overlap event ordering end to end).
        synchronize(dev)
        res.relerr = max((allreduced_relerr(ctx, A[min(i, lb - 1)], B[min(i, lb - 1)], Cb)
                          for i, Cb in checked), default=0.0)
    if hasattr(direct, "npeers"):  # IpcGather: peers mapped for the pulls
        res.extra["ipc_peers"] = direct.npeers
    if hasattr(direct, "close"):  # IpcGather: unmap the peers' buffers before anyone frees
        direct.close()
    return res
