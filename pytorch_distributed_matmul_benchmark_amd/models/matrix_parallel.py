"""``matrix_parallel`` mode: 1-D column-parallel GEMM + RCCL all-gather.

Reference: matmul_scaling_benchmark.py:167-238. A is replicated, B is split
by columns, each rank computes C_local = A @ B_local ([N, N/ws]) and the
column blocks are all-gathered into a list of ws tensors (re-allocated each
iteration, never concatenated). TFLOPS = 2N³ / t / ws per rank
("portion"), system = AVG of that, "Actual" = 2N³ / t.

Differences:
  * Q15: A comes from one seed on every rank (replicated by construction),
    and each B_local is the rank's column slice of ONE global B, so the
    gathered result is exactly A @ B and can be checked.
  * Q4: shards are padded to a uniform width (``column_shard``), so the
    all-gather is valid for any N and ws; padding columns are zero.
  * Q16: the gather target is one preallocated buffer
    ``[ws*N, shard]`` filled by ``all_gather_into_tensor`` (block r =
    C[:, r*shard:(r+1)*shard]); no per-iteration allocation and no list
    copy-out.
  * ``--allgather``: RCCL's ``all_gather_into_tensor`` (default), the direct
    P2P group (``direct``), or ``ipc``: every rank pulls the peers' blocks
    out of their C_local over xGMI peer memory with DMA-engine copies
    (parallel/ipc.py; C_local lives in IPC-exportable allocations).
  * ``overlap=True`` (parallel/overlap.py OverlapPipeline): C_local is ONE
    GEMM launch per iteration into a ring of two buffers (the reference's
    C1/C2, backup/matmul_overlap_benchmark.py:98-101); iteration i's
    all-gather runs on the high-priority comm stream while iteration i+1
    computes, and — where the planner says so — starts piece by piece as the
    GEMM's own tiles complete (W4 completion signals), the GEMM optionally on
    a CU-masked stream (``comm_cus``). Gather layout: per (ring slot, piece)
    ``[ws*rows_p, shard]``. A plan that loses to serializing runs serialized.
"""
from __future__ import annotations

import torch

from ..parallel.comm import CommStream, current_stream
from ..parallel.ipc import ipc_empty
from ..parallel.overlap import (OverlapPipeline, all_gather_now, compute_ctx, compute_stream,
                                gather_fn, ipc_buffers, make_gatherer, measured_plan,
                                pick_collective)
from ..parallel.dist import DistContext
from ..parallel.partition import column_shard
from ..utils.metrics import gemm_flops, tflops_from
from ..utils.timing import SegmentTimer, Stopwatch, synchronize, time_loop_ms
from . import independent
from .common import (ModeResult, Workload, align_ranks, gemm_fn, kernel_label, out_dtype, randn,
                     sampled_relerr, warmup, zeros_b)


def make_operands(w: Workload, ctx: DistContext):
    """(A replicated, B_local padded column shard, shard) for this rank."""
    dev, n, ws = ctx.device, w.n, ctx.world_size
    sh = column_shard(n, ws, ctx.rank, align=8)
    A = randn((n, n), w, dev, seed=10_000 + w.seed)
    Bg = randn((n, n), w, dev, seed=10_001 + w.seed, operand="B")   # the one global B
    B_local = zeros_b(n, sh.padded, w, dev)
    if sh.width:
        B_local[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
    del Bg
    return A, B_local, sh


def scaled_b(B: torch.Tensor, s: float) -> torch.Tensor:
    """``B x s`` in B's own layout (fp8: column-major, scaled through fp32; a
    power-of-two ``s`` is exact in every dtype, short of overflow)."""
    if B.dtype == torch.float8_e4m3fn:
        return (B.t().float() * s).to(B.dtype).t()
    return B * s


def assemble(gathered, n: int, ws: int) -> torch.Tensor:
    """Full [N, N] C from gather buffer(s) of shape [ws*rows, shard] (drops padding).

    ``gathered`` is one buffer or a list of per-row-chunk buffers."""
    bufs = gathered if isinstance(gathered, (list, tuple)) else [gathered]
    parts = []
    for g in bufs:
        rows = g.shape[0] // ws
        parts.append(g.view(ws, rows, -1).permute(1, 0, 2).reshape(rows, -1)[:, :n])
    return torch.cat(parts, dim=0)


def run(w: Workload, ctx: DistContext) -> ModeResult:
    ws = ctx.world_size
    if ws == 1 or not ctx.is_distributed:
        # matmul_scaling_benchmark.py:171-172 — one GPU does the whole product.
        r = independent.run(w, ctx, mode_name="matrix_parallel")
        return r
    dev, n = ctx.device, w.n
    A, B_local, sh = make_operands(w, ctx)
    # --allgather ipc: peers pull their blocks straight out of C_local, so the
    # outputs live in IPC-exportable allocations (parallel/ipc.py)
    alloc = ((lambda: ipc_empty((n, sh.padded), out_dtype(w), dev)) if ipc_buffers(w.allgather, dev)
             else (lambda: torch.empty((n, sh.padded), device=dev, dtype=out_dtype(w))))
    C_local = alloc()
    mm = gemm_fn(w, dev)
    label = kernel_label(w, A, B_local, C_local)
    flops_local = gemm_flops(n, sh.padded, n)
    flops_total = gemm_flops(n, n, n)
    extra = {"shard_cols": sh.padded, "overlap": bool(w.overlap), "allgather": w.allgather}
    units = [(A, B_local, C_local), (A, B_local, alloc())]
    plan = None
    compute, owner = compute_stream(dev, w.comm_cus) if w.overlap else (current_stream(dev), None)
    impl = w.allgather

    def gatherer(sources, comm):
        """(impl, comm object) — auto: the fastest of rccl / direct / ipc, timed here."""
        if impl == "auto":
            spread = {}
            chosen, obj, times = pick_collective(ctx, "all_gather", C_local, sources, comm=comm,
                                                 spread_out=spread)
            extra["allgather"], extra["collective_us"] = f"auto:{chosen}", times
            extra["collective_spread_us"] = spread
            return chosen, obj
        if impl == "rccl" and comm is None:
            return impl, None
        return impl, make_gatherer(impl, dev, sources, comm=comm)

    if w.overlap:
        cs = CommStream(dev)
        impl, gath = gatherer([u[2] for u in units], cs)
        g = gather_fn(impl, gath)
        probe_out = {}

        def prepare(s, e):  # the probe's scratch gather buffer (agreed before any collective)
            if e - s not in probe_out:
                probe_out[e - s] = torch.empty((ws * (e - s), sh.padded), device=dev,
                                               dtype=out_dtype(w))

        def probe(s, e):  # one piece's all-gather, into that buffer
            prepare(s, e)
            g(probe_out[e - s], units[0][2][s:e])
        # priced from this job's own GEMM and all-gather times (MAX over ranks)
        plan = measured_plan(units, ctx, "all_gather", n * sh.padded * C_local.element_size(), mm,
                             probe, native=w.backend == "native", requested=w.chunks,
                             steps=max(w.iters, 1), compute=compute, owner=owner, comm=cs,
                             piece_prepare=prepare)
        del probe_out
        extra["plan"] = plan.as_dict()

    if plan is None or not plan.overlap:
        # dim-0 concatenation [ws*N, shard] (the layout both gloo and RCCL accept);
        # block r = gathered.view(ws, N, shard)[r] = C[:, r*shard:(r+1)*shard].
        gathered = torch.empty((ws * n, sh.padded), device=dev, dtype=out_dtype(w))

        if w.overlap:  # the planner serialized: the gatherer built for it is the one
            cs = gath
        else:
            impl, cs = gatherer([C_local], None)

        def comm():
            all_gather_now(gathered, C_local, impl, cs)

        def serial_step():
            mm(A, B_local, C_local)
            comm()

        warmup(serial_step, w, ctx)
        align_ranks(ctx)
        seg = SegmentTimer(dev)
        st = current_stream(dev)
        seg.begin(st)
        for _ in range(w.iters):
            mm(A, B_local, C_local)
            seg.mark("compute", st)
            comm()
            seg.mark("comm", st)
        tot = seg.totals_ms()
        it = max(w.iters, 1)
        comp, cm = tot.get("compute", 0.0) / it, tot.get("comm", 0.0) / it
        avg = comp + cm
        full = (lambda: assemble(gathered, n, ws))
    else:
        bufs = {}

        def coll(r, p, s, e, after, done):
            if (r, p) not in bufs:
                bufs[(r, p)] = torch.empty((ws * (e - s), sh.padded), device=dev,
                                           dtype=out_dtype(w))
            g(bufs[(r, p)], units[r][2][s:e], after=after, done=done)

        operands = None
        if w.check:
            # every unit its own product: B_local x 2^(k mod 3) — exact in every
            # dtype (a power-of-two scale), and a unit's ring slot last held
            # another scale's product, so a piece gathered before its GEMM
            # rewrote the slot (or after the next one did) fails the check
            scaled = [B_local, scaled_b(B_local, 2), scaled_b(B_local, 4)]

            def operands(k):
                return A, scaled[k % 3]
        pipe = OverlapPipeline(mm, units, coll, dev, plan, per_step=1, compute=compute,
                               owner=owner, comm=cs, operands=operands)
        extra["pieces"] = len(pipe.pieces)
        extra["signalled"] = pipe.signalled
        extra["comm_cus"] = len(owner.excluded) if owner is not None else 0
        label = ("pdmb_w4_nn (completion signals)" if pipe.signalled
                 else kernel_label(w, A, B_local, C_local, shared=True))

        def finish():
            pipe.finish()
            if compute is not None:  # the timing stream joins the (masked) compute stream
                current_stream(dev).wait_stream(compute)

        warmup(lambda: (pipe.step(), finish()), w, ctx)
        align_ranks(ctx)
        sw = Stopwatch(dev)
        sw.start(current_stream(dev))
        for _ in range(w.iters):
            pipe.step()
        finish()
        sw.stop(current_stream(dev))
        avg = sw.elapsed_ms() / max(w.iters, 1)
        synchronize(dev)
        # the gathered C of the last R units, each with its own scale (check)
        gathered_units = [(pipe.slot_unit[r], [bufs[(r, p)] for p in range(len(pipe.pieces))])
                          for r in range(len(units)) if pipe.used[r]]
        k = max(1, min(w.iters, 10))
        spare = torch.empty_like(C_local)

        def gemm_only():  # same context as the pipeline's GEMMs; the ring keeps its outputs
            with compute_ctx(compute, owner):
                mm(A, B_local, spare)
            if compute is not None:
                current_stream(dev).wait_stream(compute)
        comp = time_loop_ms(gemm_only, k, 1, dev) / k
        cm = max(avg - comp, 0.0)
        pipe.close()
        full = None

    res = ModeResult(mode="matrix_parallel", n=n, world_size=ws, avg_ms=avg,
                     flops_local=flops_local, flops_total=flops_total,
                     tflops=tflops_from(flops_total, avg / 1e3) / ws,
                     compute_ms=comp, comm_ms=cm,
                     compute_only_tflops=tflops_from(flops_local, comp / 1e3),
                     kernel=label, extra=extra)
    if w.check:
        synchronize(dev)
        Bg = randn((n, n), w, dev, seed=10_001 + w.seed, operand="B")
        if full is not None:
            res.relerr = sampled_relerr(A, Bg, full())
        else:
            # every gathered piece of the last R units against ITS unit's product
            # (256 sampled rows: a stale piece spans >= 256 rows of the 4096+)
            Bd = Bg.double()
            res.relerr = max((sampled_relerr(A, Bd * float(2 ** (k % 3)), assemble(pieces, n, ws),
                                             rows=256)
                              for k, pieces in gathered_units), default=float("inf"))
            extra["checked_units"] = [k for k, _ in gathered_units]
    gatherer = cs if (plan is None or not plan.overlap) else gath
    if hasattr(gatherer, "npeers"):  # IpcGather: peers mapped for the pulls
        res.extra["ipc_peers"] = gatherer.npeers
    if hasattr(gatherer, "close"):  # IpcGather: unmap the peers' buffers before anyone frees
        gatherer.close()
    return res
