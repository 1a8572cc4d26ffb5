"""``ring_parallel`` mode: all-gather-GEMM over an xGMI ring (sequence-parallel
column-parallel GEMM), the block-rotation structure of ring attention.

Not in the reference. Its only "split one big op" strategy is
matrix_parallel (matmul_scaling_benchmark.py:167-238), which REPLICATES A on
every rank and then all-gathers C. SURVEY §5 ("Long-context / sequence
parallelism") names the ring all-gather-GEMM as the analogue worth building.
Here A is not replicated; it is row-sharded like a sequence shard:

  * rank r owns A rows ``R_r`` (``column_shard`` of the N rows, 256-aligned so
    every hop's GEMM is whole 256-row tiles) and B columns ``S_r``
    (matrix_parallel's column shard);
  * it computes C[:, S_r] = A @ B[:, S_r] — matrix_parallel's local product —
    in ws row blocks, using BOTH directions of the ring: each A block is cut
    into a top and a bottom half; tops travel clockwise (r -> r+1), bottoms
    counter-clockwise (r -> r-1). At hop s the rank multiplies the top half
    of rank (r - s)'s block and the bottom half of rank (r + s)'s block while,
    on the high-priority comm stream, it forwards both halves and receives
    the next two (one batched isend/irecv group of 4 transfers per hop);
  * so compute of hop s overlaps the transfers for hop s+1, and each hop
    moves N²/(2 ws) elements over EACH of the two xGMI links to the ring
    neighbours (a one-directional ring moves N²/ws over one link: per-link
    bound). A and C stay sharded (N²/ws elements each per rank),
    so per-rank memory does not grow with N² as matrix_parallel's
    replicated A and gathered C do.

Event protocol (two receive buffers per direction; hop 0 reads the rank's
own block):

    comm hop s : wait(last GEMM issued) → send top_s → r+1, recv Rt[(s+1)%2] ← r-1,
                 send bot_s → r-1, recv Rb[(s+1)%2] ← r+1 → record(recv_done[s])
    compute s+1: wait(recv_done[s]) → GEMM(Rt[(s+1)%2]), GEMM(Rb[(s+1)%2])

Waiting for the most recently issued GEMM before each hop guarantees that
the buffers being overwritten (read by hop s-1's GEMMs) are no longer in
use; the GEMMs of hop s run concurrently with the hop's transfers.

TFLOPS follows matrix_parallel: "portion" = 2N³ / t / ws per rank, system =
AVG of that, Actual = 2N³ / t.
"""
from __future__ import annotations

import torch

from ..ops import gemm
from ..parallel.comm import current_stream
from ..parallel.overlap import BidirRing
from ..parallel.dist import DistContext
from ..parallel.partition import column_shard
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import Stopwatch, synchronize, time_loop_ms
from . import independent
from .common import (ModeResult, Workload, align_ranks, gemm_fn, kernel_label, out_dtype, randn,
                     sampled_relerr, warmup, zeros_b)

ROW_ALIGN = 512  # two GEMM tiles: each half-block product is whole 256-row tiles


def make_operands(w: Workload, ctx: DistContext):
    """(A_local [rows_padded, N] zero-padded row block, B_local [N, cols_padded],
    row shard, column shard). A and B are slices of ONE global A / B (seeded
    identically on every rank), so the result is checkable against A @ B."""
    dev, n, ws, r = ctx.device, w.n, ctx.world_size, ctx.rank
    rs = column_shard(n, ws, r, align=ROW_ALIGN)
    cs = column_shard(n, ws, r, align=8)
    Ag = randn((n, n), w, dev, seed=10_000 + w.seed)
    A_local = torch.zeros((rs.padded, n), device=dev, dtype=w.dtype)
    if rs.width:
        A_local[:rs.width].copy_(Ag[rs.start:rs.stop])
    del Ag
    Bg = randn((n, n), w, dev, seed=10_001 + w.seed, operand="B")
    B_local = zeros_b(n, cs.padded, w, dev)
    if cs.width:
        B_local[:, :cs.width].copy_(Bg[:, cs.start:cs.stop])
    del Bg
    return A_local, B_local, rs, cs


def assemble_rows(C_local: torch.Tensor, n: int, ws: int, rows_padded: int) -> torch.Tensor:
    """C[:, S_r] ([N, cols_padded]) from the per-source row blocks of ``C_local``
    ([ws*rows_padded, cols_padded], block j = rows of rank j's A), padding dropped."""
    parts = []
    for j in range(ws):
        sh = column_shard(n, ws, j, align=ROW_ALIGN)
        parts.append(C_local[j * rows_padded: j * rows_padded + sh.width])
    return torch.cat(parts, dim=0)


def run(w: Workload, ctx: DistContext) -> ModeResult:
    ws = ctx.world_size
    if ws == 1 or not ctx.is_distributed:
        return independent.run(w, ctx, mode_name="ring_parallel")
    dev, n, r = ctx.device, w.n, ctx.rank
    A_local, B_local, rs, csh = make_operands(w, ctx)
    rp = rs.padded
    C_local = torch.empty((ws * rp, csh.padded), device=dev, dtype=out_dtype(w))
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A_local[:rp // 2], B_local, C_local[:rp // 2], shared=True)
    compute = current_stream(dev)
    ring = BidirRing(A_local, rp, r, ws, dev)

    def step():
        with gemm.shared_device():  # the hops' transfers run beside these GEMMs
            ring.step(mm, B_local, C_local, compute)

    warmup(step, w, ctx)
    align_ranks(ctx)
    sw = Stopwatch(dev)
    sw.start(compute)
    for _ in range(w.iters):
        step()
    sw.stop(compute)
    avg = sw.elapsed_ms() / max(w.iters, 1)
    synchronize(dev)

    def gemms_only():
        for j in range(ws):
            mm(A_local, B_local, C_local[j * rp:(j + 1) * rp])

    k = max(1, min(w.iters, 10))
    Cref = C_local.clone() if w.check else None  # the timed loop's result, before re-timing
    comp = time_loop_ms(gemms_only, k, 1, dev) / k
    cm = max(avg - comp, 0.0)
    flops_local = gemm_flops(ws * rp, csh.padded, n)
    flops_total = gemm_flops(n, n, n)
    res = ModeResult(mode="ring_parallel", n=n, world_size=ws, avg_ms=avg,
                     flops_local=flops_local, flops_total=flops_total,
                     tflops=tflops_from(flops_total, avg / 1e3) / ws,
                     compute_ms=comp, comm_ms=cm,
                     compute_only_tflops=tflops_from(flops_local, comp / 1e3),
                     kernel=label,
                     extra={"shard_rows": rp, "shard_cols": csh.padded, "hops": ws - 1, "directions": 2,
                            "overlap": True})
    if w.check:
        synchronize(dev)
        Cc = assemble_rows(Cref, n, ws, rp)
        Ag = randn((n, n), w, dev, seed=10_000 + w.seed)
        res.relerr = sampled_relerr(Ag, B_local, Cc)
    return res
