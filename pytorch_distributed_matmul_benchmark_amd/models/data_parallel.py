"""backup ``data_parallel`` mode: full N×N GEMM per rank + all-reduce of the
full N×N output.

Reference: backup/matmul_distributed_benchmark.py:66-110 — serialized
compute/comm events with host syncs; TFLOPS from compute time only;
returns (t_total, tflops, t_comm); the runner prints compute / comm /
overhead % and an inverted "scaling efficiency" (:252-258).
Here the same quantities come from stream events (no in-loop host sync),
and efficiency is compute / total (100 % = comm free).
"""
from __future__ import annotations

import torch
from ..parallel.comm import current_stream
from ..parallel.ipc import ipc_empty
from ..parallel.overlap import all_reduce_now, make_gatherer
from ..parallel.dist import DistContext
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import SegmentTimer
from .common import (ModeResult, Workload, align_ranks, allreduced_relerr, gemm_fn, kernel_label,
                     out_dtype, randn, warmup)


def run(w: Workload, ctx: DistContext) -> ModeResult:
    dev, n, ws = ctx.device, w.n, ctx.world_size
    impl = "rccl" if w.allreduce == "auto" else w.allreduce  # auto: batch_parallel only
    A = randn((n, n), w, dev, seed=2 * (w.seed + ctx.rank))
    B = randn((n, n), w, dev, seed=2 * (w.seed + ctx.rank) + 1, operand="B")
    # --allreduce ipc: peers pull chunks straight out of C (IPC-exportable allocation)
    C = (ipc_empty((n, n), out_dtype(w), dev) if impl == "ipc"
         else torch.empty((n, n), device=dev, dtype=out_dtype(w)))
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A, B, C)
    distributed = ctx.is_distributed
    # the collective's comm object: a CommStream (direct) or an IpcGather (ipc)
    direct = make_gatherer(impl, dev, [C]) if impl != "rccl" and distributed else None

    def step():
        mm(A, B, C)
        if distributed:
            all_reduce_now(C, impl, direct)

    warmup(step, w, ctx)
    align_ranks(ctx)
    seg = SegmentTimer(dev)
    st = current_stream(dev)
    seg.begin(st)
    for _ in range(w.iters):
        mm(A, B, C)
        seg.mark("compute", st)
        if distributed:
            all_reduce_now(C, impl, direct)
        seg.mark("comm", st)
    tot = seg.totals_ms()
    it = max(w.iters, 1)
    comp, comm = tot.get("compute", 0.0) / it, tot.get("comm", 0.0) / it
    flops = gemm_flops(n, n, n)
    res = ModeResult(mode="data_parallel", n=n, world_size=ws, avg_ms=comp + comm,
                     flops_local=flops, flops_total=flops * ws,
                     tflops=tflops_from(flops, comp / 1e3), compute_ms=comp, comm_ms=comm,
                     compute_only_tflops=tflops_from(flops, comp / 1e3), kernel=label,
                     extra={"allreduce": impl})
    if w.check:
        res.relerr = allreduced_relerr(ctx, A, B, C)
    if hasattr(direct, "close"):  # IpcGather: unmap the peers' buffers before anyone frees
        direct.close()
    return res
