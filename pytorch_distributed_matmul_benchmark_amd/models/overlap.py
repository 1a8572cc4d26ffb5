"""backup overlap family: ``no_overlap`` | ``overlap`` | ``pipeline``.

Reference: backup/matmul_overlap_benchmark.py:36-278. Every iteration is a
full N×N GEMM whose output is all-reduced (a DP gradient stand-in):
  * no_overlap (:36-91): GEMM → sync → all_reduce → sync, serialized.
  * overlap (:93-180): two A/B/C buffer sets, a compute and a comm stream,
    all-reduce of buffer i%2 while computing the other one.
  * pipeline (:182-278): 3 buffer sets / 3 compute streams, async handles
    waited FIFO once 3 are outstanding.
Each then re-measures 10 compute-only iterations for a TFLOPS figure that
the reference computes but never prints (Q9).

The reference's overlap has a data race (Q7): the collective is ordered
after the comm stream only, not after the GEMM that writes the buffer, and
the handle is dropped, so the next GEMM may overwrite a buffer that is
still being reduced; pipeline issues its all-reduce on the default stream
while the GEMMs run on three others. Here both are an event-ordered ring
of ``depth`` buffers (overlap: 2, pipeline: 3):

    compute: wait done[i % d] → GEMM → C[i % d]; record ready[i % d]
    comm   : wait ready[i % d] → RCCL all_reduce(C[i % d]); record done[i % d]

One compute stream: on MI355X a single 16k GEMM already fills all 256 CUs
(4096 256×256 tiles), so extra compute streams add nothing but contention;
the ring depth is what lets compute run ahead of the comm stream.
Reported: per-iteration wall time, "Actual TFLOPS" = 2N³ / t_iter, and the
compute-only TFLOPS.
"""
from __future__ import annotations

import torch

from ..ops import gemm
from ..parallel.comm import CommStream, current_stream, new_event
from ..parallel.dist import DistContext
from ..parallel.ipc import ipc_empty
from ..parallel.overlap import all_reduce_now, make_gatherer, reduce_fn
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import Stopwatch, synchronize, time_loop_ms
from .common import (ModeResult, Workload, align_ranks, allreduced_relerr, gemm_fn, kernel_label,
                     out_dtype, randn, warmup)

DEPTH = {"no_overlap": 1, "overlap": 2, "pipeline": 3}


def run(w: Workload, ctx: DistContext, mode: str = "overlap", depth: int = None) -> ModeResult:
    """``depth`` overrides the ring depth (reference ``pipeline_depth``,
    backup/matmul_overlap_benchmark.py:184); default 1 / 2 / 3 by mode."""
    if mode not in DEPTH:
        raise ValueError(f"unknown overlap mode {mode!r}")
    dev, n, ws = ctx.device, w.n, ctx.world_size
    impl = "rccl" if w.allreduce == "auto" else w.allreduce  # auto: batch_parallel only
    depth = DEPTH[mode] if depth is None else max(1, int(depth))
    As = [randn((n, n), w, dev, seed=100 * (w.seed + ctx.rank) + 2 * i) for i in range(depth)]
    Bs = [randn((n, n), w, dev, seed=100 * (w.seed + ctx.rank) + 2 * i + 1, operand="B") for i in range(depth)]
    # --allreduce ipc: peers pull chunks straight out of the C ring (IPC-exportable)
    Cs = [ipc_empty((n, n), out_dtype(w), dev) if impl == "ipc"
          else torch.empty((n, n), device=dev, dtype=out_dtype(w)) for _ in range(depth)]
    mm = gemm_fn(w, dev)
    distributed = ctx.is_distributed
    label = kernel_label(w, As[0], Bs[0], Cs[0], shared=depth > 1 and distributed)
    compute = current_stream(dev)
    # the collective's comm object: the CommStream, or (ipc on GPUs) an IpcGather
    # with every ring buffer registered
    cs = CommStream(dev)
    comm = make_gatherer(impl, dev, Cs, comm=cs) if distributed and impl != "rccl" else cs

    used = [True] + [False] * (depth - 1)
    if depth == 1 or not distributed:
        def run_iters(k):
            for _ in range(k):
                mm(As[0], Bs[0], Cs[0])
                if distributed:
                    all_reduce_now(Cs[0], impl, comm)
        finish = (lambda: None)
    else:
        ar = reduce_fn(impl, comm)
        ready = [new_event(dev) for _ in range(depth)]
        done = [new_event(dev) for _ in range(depth)]
        used[0] = False
        counter = [0]

        def run_iters(k):
            for _ in range(k):
                i = counter[0] % depth
                counter[0] += 1
                if used[i] and compute is not None:
                    compute.wait_event(done[i])   # WAR: buffer's previous reduce finished
                with gemm.shared_device():  # earlier buffers' all-reduces run beside it
                    mm(As[i], Bs[i], Cs[i])
                ready[i].record(compute)
                ar(Cs[i], after=ready[i], done=done[i])
                used[i] = True

        def finish():
            if compute is not None:
                for i in range(depth):
                    if used[i]:
                        compute.wait_event(done[i])

    warmup(lambda: run_iters(1), w, ctx)
    finish()
    # Compute-only time (backup/matmul_overlap_benchmark.py:77-89 re-measures 10
    # GEMM-only iterations), taken before the timed loop so the loop's reduced
    # buffers stay intact for --check.
    synchronize(dev)
    k = max(1, min(w.iters, 10))
    comp = time_loop_ms(lambda: mm(As[0], Bs[0], Cs[0]), k, 0, dev) / k
    align_ranks(ctx)
    sw = Stopwatch(dev)
    sw.start(compute)
    run_iters(w.iters)
    finish()
    sw.stop(compute)
    avg = sw.elapsed_ms() / max(w.iters, 1)
    flops = gemm_flops(n, n, n)
    res = ModeResult(mode=mode, n=n, world_size=ws, avg_ms=avg, flops_local=flops,
                     flops_total=flops * ws, tflops=tflops_from(flops, avg / 1e3),
                     compute_ms=comp, comm_ms=max(avg - comp, 0.0),
                     compute_only_tflops=tflops_from(flops, comp / 1e3), kernel=label,
                     extra={"depth": depth})
    if w.check:
        # Each ring buffer's last GEMM was all-reduced before the loop ended:
        # C[i] must equal Σ_ranks A_r[i] @ B_r[i] (a write-while-reducing race,
        # reference Q7, shows up here).
        synchronize(dev)
        res.relerr = max(allreduced_relerr(ctx, As[i], Bs[i], Cs[i])
                         for i in range(depth) if used[i] or i == 0)
    if hasattr(comm, "close"):  # IpcGather: unmap the peers' buffers before anyone frees
        comm.close()
    return res
