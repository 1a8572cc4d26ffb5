#!/usr/bin/env python3
"""Driver benchmark: whole-node TFLOPS of the 16k×16k bf16 GEMM on N MI355X GPUs.

Metric and config are BASELINE.json's headline: "TFLOPS (whole node) +
scaling efficiency, 16k×16k bf16 GEMM at 1/2/4/8 GPUs" — the reference's
``matmul_benchmark.py`` / ``matmul_scaling_benchmark.py --mode independent``
16384² bf16 number (README.md:43-44: ~140 TFLOPS on 1 RTX 6000 Ada, ~294 on 2).

One "step" = one 16384×16384×16384 bf16 GEMM per GPU on the hand-written
gfx950 MFMA kernel (``--mode independent``, weak scaling: per-GPU work is
fixed as N grows). ``--mode batch_parallel`` (bmm + RCCL all-reduce of the
output) and ``--mode matrix_parallel`` (column-sharded B + RCCL all-gather,
strong scaling) are available too. W untimed warmup steps, then exactly K
timed steps bracketed by barrier + synchronize on both sides; the max over
ranks of the elapsed wall time is the step time; rank 0 prints one JSON line.

After the headline measurement (which is what ``value`` reports) the same
process also times the reference's other two scaling modes — batch_parallel
(matmul_scaling_benchmark.py:106-165) and matrix_parallel (:167-238), each
serialized as in the reference and with the collective overlapped on the
comm stream (parallel/overlap.py OverlapPipeline: whole GEMMs, a ring of
outputs, pieces started by the GEMM's own completion signals; the plan is
in the line) — for ``--extra-steps`` steps each, and reports them under
``"modes"`` in the same JSON line, so one launch at N GPUs yields the
BASELINE configs 3-5 (``--extra-steps 0`` skips them). Each secondary mode
warms up for at least ``--extra-warmup-ms`` of GPU time and is compared
with a same-shape reference run on rank 0 alone just before its family
(batch: the bmm of the local batch; matrix: the whole N x N GEMM), so its
``scaling_efficiency`` isolates communication from clock drift.

Verifiability: the line carries the process-group backend, the world size
the group saw, the RCCL version, the collective self-test result (run
before any timing), per-rank TFLOPS min / max, the serialized modes'
compute / comm split, and per-mode median GFX clock and power (amdsmi, 5 ms
poll, with the sample counts).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without torchrun self-launches N ranks (a child
``torch.distributed.run``, started before anything touches the GPU; the GPU
count comes from sysfs / amdsmi, never HIP) and exits with its code; under torchrun, ``WORLD_SIZE != --gpus`` is an error. At N > 1
the job also times the headline GEMM on rank 0 alone (others at a barrier)
and reports ``scaling_efficiency = value / (N x single_gpu_tflops)`` — the
1 -> N curve's efficiency from one launch. Every mode's setup is agreed
across ranks (a setup failure becomes an ``"error"`` entry, no hang); a
failure inside a timed region exits that rank at once, so torchrun tears the
job down in seconds (fault injection: ``PDMB_BENCH_FAULT=rank:mode:phase``).
"""
from __future__ import annotations

import argparse
import contextlib
import gc
import json
import math
import os
import signal
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.comm import CommStream  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.ipc import ipc_empty  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.dist import (  # noqa: E402
    DistContext, all_ok, barrier, cleanup_distributed, gather_scalars, reduce_scalar,
    setup_distributed, verify_collectives)
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import (  # noqa: E402
    BidirRing, OverlapPipeline, all_gather_now, all_reduce_now, compute_ctx, gather_fn, make_gatherer,
    ipc_buffers, measured_plan, pick_collective, reduce_fn, compute_stream)
from pytorch_distributed_matmul_benchmark_amd.parallel.partition import (  # noqa: E402
    column_shard, global_batch, local_batch)
from pytorch_distributed_matmul_benchmark_amd.utils import testhooks  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.utils.telemetry import (  # noqa: E402
    ClockSampler, visible_gpus)

# Reference numbers (README.md:43-46): whole-system TFLOPS at 16k bf16.
BASELINE_TFLOPS = {"independent": {1: 140.0, 2: 294.0},
                   "batch_parallel": {1: 140.0, 2: 237.0},
                   "matrix_parallel": {1: 140.0, 2: 141.0}}
METRIC = "TFLOPS (whole node) + scaling efficiency, 16k×16k bf16 GEMM at 1/2/4/8 GPUs"
DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
          "float8_e4m3fn": torch.float8_e4m3fn}


def collective_impl(flag, overlap: bool) -> str:
    """``--allreduce`` / ``--allgather`` as given, or by default: RCCL for the
    serialized modes (the reference's NCCL call, matmul_scaling_benchmark.py:
    150 / :221, so those numbers stay reference-comparable) and ``auto`` for the
    overlapped ones (the fastest of RCCL / direct / the peer-memory pull,
    timed on the job's own ranks: the MI355X-native schedule)."""
    if flag:
        return flag
    return "auto" if overlap else "rccl"


class Workload:
    """Operands + one timed ``step()`` of a scaling mode on this rank.

    ``batch`` (independent only): GEMMs per step (a bmm), the rank-0-alone
    reference of batch_parallel's local batch."""

    def __init__(self, a, ctx, mode: str, overlap: bool, batch: int = 1,
                 test_corrupt_rank: int | None = None):
        self.ctx, self.mode, self.overlap = ctx, mode, overlap
        # tests only (the per-mode check's negative control): verify() damages
        # one checked output on this rank before comparing; never set by main()
        self._test_corrupt_rank = test_corrupt_rank
        self.cuda = ctx.device.type == "cuda"
        self.dt = DTYPES[a.dtype]
        self.backend = a.backend
        dev, n, ws, dt = ctx.device, a.size, ctx.world_size, self.dt
        odt = gemm.out_dtype(dt)  # fp8 operands write a bf16 C
        self._g = torch.Generator(device=dev)
        flop_gemm = 2.0 * n * n * n
        overlap = overlap and ws > 1
        self.finish = lambda: None       # issues what a pipelined step left pending + joins
        self.split = None                # serialized modes: [(ev0, ev_compute, ev_comm)] per timed step
        self.recording = False
        self.plan = None
        self.coll_choice = None          # --allreduce / --allgather auto: the measured choice
        self.pipe = None
        self.step = None                 # set below, or by _pipeline
        self._closers = []               # collective teardown (IpcGather.close), run by close()
        self._negate = []                # verify(): operands whose sign the check step flips
        self._targets = lambda: []       # verify(): what the check step's outputs must satisfy
        self._fallback_gathered = {}     # serialized fallback's all-gather outputs, by ring slot
        comp = torch.cuda.current_stream(dev) if self.cuda else None
        self._mask = None
        if overlap and self.cuda and a.comm_cus > 0 and mode in ("batch_parallel", "matrix_parallel",
                                                                 "ring_parallel"):
            # GEMMs on a CU-masked stream, RCCL gets the free CUs at once
            comp, self._mask = compute_stream(dev, a.comm_cus)
        self.comp = comp

        if mode == "independent":
            shape = (batch, n, n) if batch > 1 else (n, n)
            A = self._rnd(*shape, seed=2 * ctx.rank)
            B = self._rnd(*shape, seed=2 * ctx.rank + 1, b=True)
            C = torch.empty(*shape, device=dev, dtype=odt)
            self.kernel = self._label(A, B, C)

            def step():
                self._mm(A, B, C)
            self._negate = [A]
            self._targets = lambda: ([("gemm", A[i], B[i], C[i]) for i in sorted({0, batch - 1})]
                                     if batch > 1 else [("gemm", A, B, C)])
            self.flops = flop_gemm * ws * batch
            self.global_batch, self.parallelism = ws * batch, f"independent{ws}"
        elif mode == "batch_parallel":
            lb, gb = local_batch(ws), global_batch(ws)
            A = self._rnd(lb, n, n, seed=2 * ctx.rank)
            B = self._rnd(lb, n, n, seed=2 * ctx.rank + 1, b=True)
            # --allreduce ipc / auto: peers may pull chunks straight out of C
            # (IPC-exportable allocations)
            ar_impl = collective_impl(a.allreduce, overlap)
            alloc = ((lambda *shape: ipc_empty(shape, odt, dev)) if ipc_buffers(ar_impl, dev)
                     else (lambda *shape: torch.empty(*shape, device=dev, dtype=odt)))
            C = alloc(lb, n, n)
            self.kernel = self._label(A, B, C)
            self._negate = [A]
            if overlap:
                # ring over the batch's own outputs; one element: a second C (reference C1/C2)
                units = ([(A[b], B[b], C[b]) for b in range(lb)] if lb >= 2 else
                         [(A[0], B[0], C[0]), (A[0], B[0], alloc(n, n))])
                cs = CommStream(dev)
                srcs = [C] + ([units[1][2]] if lb == 1 else [])
                impl, peer = self._collective(ar_impl, "all_reduce", units[0][2], srcs, cs)
                self._closers.append(getattr(peer, "close", None))
                ar = reduce_fn(impl, peer)

                def coll(r, p, s, e, after, done):
                    ar(units[r][2][s:e], after=after, done=done)
                self._pipeline(a, units, coll, lb, "all_reduce", n * n * C.element_size(), cs, peer,
                               probe=lambda s, e: ar(units[0][2][s:e]), impl=impl)
                self._targets = lambda: [("reduce", *units[r]) for r in self._last_slots(lb)]
            else:
                self._serial_split()
                impl, cs = self._collective(ar_impl, "all_reduce", C[0], [C], None)
                self._closers.append(getattr(cs, "close", None))

                def step():
                    self._seg(0)
                    self._mm(A, B, C)
                    self._seg(1)
                    if ws > 1:
                        all_reduce_now(C, impl, cs)
                    self._seg(2)
                self._targets = lambda: [("reduce", A[b], B[b], C[b]) for b in sorted({0, lb - 1})]
            self.flops = flop_gemm * gb
            self.global_batch, self.parallelism = gb, f"dp{ws}"
        elif mode == "matrix_parallel":
            sh = column_shard(n, ws, ctx.rank, align=8)
            A = self._rnd(n, n, seed=10_000)
            Bg = self._rnd(n, n, seed=10_001, b=True)
            Bl = (torch.zeros(sh.padded, n, device=dev, dtype=dt).t() if dt == gemm.FP8
                  else torch.zeros(n, sh.padded, device=dev, dtype=dt))
            Bl[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
            del Bg
            # --allgather ipc / auto: peers may pull their blocks out of Cl over
            # xGMI peer memory, so the outputs live in IPC-exportable allocations
            ag_impl = collective_impl(a.allgather, overlap)
            alloc = ((lambda: ipc_empty((n, sh.padded), odt, dev)) if ipc_buffers(ag_impl, dev)
                     else (lambda: torch.empty(n, sh.padded, device=dev, dtype=odt)))
            Cl = alloc()
            self.kernel = self._label(A, Bl, Cl)
            self._negate = [A]
            if overlap:
                units = [(A, Bl, Cl), (A, Bl, alloc())]
                cs = CommStream(dev)
                impl, gath = self._collective(ag_impl, "all_gather", Cl, [u[2] for u in units], cs)
                self._closers.append(getattr(gath, "close", None))
                g = gather_fn(impl, gath)
                self._gathered = {}

                def coll(r, p, s, e, after, done):
                    key = (r, p)
                    if key not in self._gathered:
                        self._gathered[key] = torch.empty(ws * (e - s), sh.padded, device=dev,
                                                          dtype=odt)
                    g(self._gathered[key], units[r][2][s:e], after=after, done=done)
                probe_out = {}

                def prepare(s, e):  # the probe's scratch gather buffer (agreed before any collective)
                    if e - s not in probe_out:
                        probe_out[e - s] = torch.empty(ws * (e - s), sh.padded, device=dev, dtype=odt)

                def probe(s, e):  # one piece's all-gather into that buffer
                    prepare(s, e)
                    g(probe_out[e - s], units[0][2][s:e])
                self._pipeline(a, units, coll, 1, "all_gather", n * sh.padded * Cl.element_size(),
                               cs, gath, probe=probe, impl=impl, prepare=prepare)
                probe_out.clear()

                def targets():
                    out = []
                    for r in self._last_slots(1):
                        out.append(("gemm", A, Bl, units[r][2]))
                        if self.pipe is not None:
                            out += [("gather", units[r][2][s:e], self._gathered[(r, p)])
                                    for p, (s, e) in enumerate(self.pipe.pieces)]
                        elif r in self._fallback_gathered:
                            out.append(("gather", units[r][2], self._fallback_gathered[r]))
                    return out
                self._targets = targets
            else:
                gathered = torch.empty(ws * n, sh.padded, device=dev, dtype=odt)
                impl, cs = self._collective(ag_impl, "all_gather", Cl, [Cl], None)
                self._closers.append(getattr(cs, "close", None))
                self._serial_split()

                def step():
                    self._seg(0)
                    self._mm(A, Bl, Cl)
                    self._seg(1)
                    if ws > 1:
                        all_gather_now(gathered, Cl, impl, cs)
                    self._seg(2)
                self._targets = lambda: [("gemm", A, Bl, Cl)] + ([("gather", Cl, gathered)] if ws > 1
                                                                  else [])
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"tp{ws}"
        elif mode == "ring_parallel":
            # Opt-in (not timed by default): all-gather-GEMM over both ring
            # directions, models/ring_parallel.py. A half-blocks rotate by P2P
            # behind each hop's GEMMs.
            rs, sh = column_shard(n, ws, ctx.rank, align=512), column_shard(n, ws, ctx.rank, align=8)
            A = self._rnd(n, n, seed=10_000)
            Al = torch.zeros(rs.padded, n, device=dev, dtype=dt)
            Al[:rs.width].copy_(A[rs.start:rs.stop])
            del A
            Bg = self._rnd(n, n, seed=10_001, b=True)
            Bl = (torch.zeros(sh.padded, n, device=dev, dtype=dt).t() if dt == gemm.FP8
                  else torch.zeros(n, sh.padded, device=dev, dtype=dt))
            Bl[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
            del Bg
            rp = rs.padded
            Cl = torch.empty(ws * rp, sh.padded, device=dev, dtype=odt)
            self.kernel = self._label(Al[:rp // 2], Bl, Cl[:rp // 2], shared=True)
            ring = BidirRing(Al, rp, ctx.rank, ws, dev)

            def step():
                # the hops' transfers run beside these GEMMs: shared device, and
                # on the (possibly CU-masked) compute stream the ring's events
                # are recorded on, joined back to the timing stream after
                with compute_ctx(self.comp, self._mask):
                    ring.step(self._mm, Bl, Cl, self.comp)
                self._join()
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"ring{ws}"
        else:
            raise ValueError(mode)
        if self.step is None:
            self.step = step

    # -- collectives -------------------------------------------------------------
    def _collective(self, impl, kind, t, sources, cs):
        """(implementation, comm object) for ``--allreduce`` / ``--allgather``
        ``impl``: ``auto`` times RCCL, the direct P2P exchange and the
        peer-memory pull on this job's ranks and keeps the fastest
        (parallel/overlap.py pick_collective; the times go into the JSON as
        ``collective``); otherwise the named one (``rccl`` on the current
        stream needs no object unless an overlap's comm stream is given)."""
        ws, dev = self.ctx.world_size, self.ctx.device
        if ws <= 1:
            return ("rccl" if impl == "auto" else impl), cs
        if impl == "auto":
            spread = {}
            impl, obj, times = pick_collective(self.ctx, kind, t, sources, comm=cs, spread_out=spread)
            self.coll_choice = {"kind": kind, "chosen": impl, "us": times, "spread_us": spread}
            if impl == "ipc":  # which pull engine ran (parallel/ipc.py PDMB_IPC_ENGINE)
                self.coll_choice["ipc_engine"] = getattr(obj, "engine", None)
            return impl, obj
        if impl == "rccl" and cs is None:
            return impl, None
        obj = make_gatherer(impl, dev, sources, comm=cs)
        if impl == "ipc" and hasattr(obj, "engine"):
            self.coll_choice = {"kind": kind, "chosen": impl, "us": None, "ipc_engine": obj.engine}
        return impl, obj

    # -- overlap ---------------------------------------------------------------
    def _pipeline(self, a, units, coll, per_step, kind, payload, cs, gath=None, probe=None,
                  impl=None, prepare=None):
        """The overlapped step: plan (parallel/overlap.py measured_plan: this
        job's own GEMM and collective times, MAX over ranks; ``probe(s, e)``
        issues one collective of rows [s, e) of ring slot 0), then an
        OverlapPipeline, or the serialized step when the plan says overlap loses."""
        A, B, C = units[0]
        self.plan = measured_plan(units, self.ctx, kind, payload, self._mm, probe,
                                  native=self.backend == "native", requested=a.chunks,
                                  steps=max(a.extra_steps, 1), compute=self.comp,
                                  owner=self._mask, comm=cs, piece_prepare=prepare)
        if not self.plan.overlap:  # the planner refuses a losing overlap: serialize
            self.step = self._serial_fallback(units, per_step, kind, impl, gath)
            return
        self.pipe = OverlapPipeline(self._mm, units, coll, self.ctx.device, self.plan,
                                    per_step=per_step, compute=self.comp, owner=self._mask, comm=cs)
        self.kernel = ("pdmb_w4_nn (completion signals)" if self.pipe.signalled
                       else self._label(A, B, C, shared=True))

        def finish():
            self.pipe.finish()
            self._join()
        self.step = self.pipe.step
        self.finish = finish

    def _serial_fallback(self, units, per_step, kind, impl, gath=None):
        """The serialized step over the same units (collective on the current stream)."""
        ws, dev = self.ctx.world_size, self.ctx.device
        gathered = self._fallback_gathered
        cs = gath if gath is not None else (CommStream(dev) if impl != "rccl" else None)

        def step():
            for r in range(per_step):
                Ar, Br, Cr = units[r]
                self._mm(Ar, Br, Cr)
                if ws <= 1:
                    continue
                if kind == "all_reduce":
                    all_reduce_now(Cr, impl, cs)
                else:
                    if r not in gathered:
                        gathered[r] = torch.empty(ws * Cr.shape[0], Cr.shape[1], device=dev,
                                                  dtype=Cr.dtype)
                    all_gather_now(gathered[r], Cr, impl, cs)
        return step

    # -- serialized compute / comm split ------------------------------------------
    def _serial_split(self):
        self.split = []

    def _seg(self, i):
        if self.split is None or not self.recording:
            return
        if i == 0:
            self.split.append([])
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
        else:
            e = time.perf_counter()
        self.split[-1].append(e)

    def split_ms(self):
        """(compute_ms, comm_ms) per step of the last timed region, or (None, None)."""
        if not self.split:
            return None, None
        comp = comm = 0.0
        for e0, e1, e2 in self.split:
            if self.cuda:
                comp += e0.elapsed_time(e1)
                comm += e1.elapsed_time(e2)
            else:
                comp += (e1 - e0) * 1e3
                comm += (e2 - e1) * 1e3
        k = len(self.split)
        return comp / k, comm / k

    # -- operands / kernels ----------------------------------------------------
    def _rnd(self, *shape, seed, b=False):
        """N(0,1) operand; fp8: rounded to e4m3 (scale 1), a B operand column-major."""
        self._g.manual_seed(seed)
        if self.dt != gemm.FP8:
            return torch.randn(*shape, generator=self._g, device=self.ctx.device, dtype=self.dt)
        x = torch.randn(*shape, generator=self._g, device=self.ctx.device, dtype=torch.float32)
        if b:
            return x.transpose(-1, -2).contiguous().to(gemm.FP8).transpose(-1, -2)
        return x.to(gemm.FP8)

    def _mm(self, A, B, out):
        if self.dt == gemm.FP8 and self.cuda and self.backend == "torch":
            one = torch.ones((), device=A.device)
            if A.dim() == 3:
                for i in range(A.shape[0]):
                    torch._scaled_mm(A[i], B[i], scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                     out=out[i])
                return out
            return torch._scaled_mm(A, B, scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                    out=out)
        if (self.backend == "torch" or not self.cuda) and self.dt != gemm.FP8:
            return torch.matmul(A, B, out=out)
        return gemm.matmul(A, B, out=out)

    def _join(self):
        """The timing (current) stream waits for the masked compute stream."""
        if self._mask is not None:
            torch.cuda.current_stream(self.ctx.device).wait_stream(self.comp)

    def _label(self, A, B, C, shared=False):
        """The kernel the step's GEMMs run (shared: beside collectives, as
        compute_ctx / the ring issue them, under gemm.shared_device)."""
        if not self.cuda:
            return "torch.matmul(cpu)"
        if self.backend != "native":
            return "hipBLASLt"
        with (gemm.shared_device() if shared else contextlib.nullcontext()):
            return gemm.kernel_for(A, B, C)

    def _sync(self):
        if self.cuda:
            torch.cuda.synchronize(self.ctx.device)

    def warm(self, warmup: int, warmup_ms: float = 0.0) -> float:
        """``warmup`` untimed steps, then more until at least ``warmup_ms`` of wall
        time has run (GPU only; the count is agreed across ranks, MAX, so ranks
        stepping collectives stay in lock-step). Returns the warm-up ms."""
        t0 = time.perf_counter()
        for _ in range(warmup):
            self.step()
        self.finish()
        self._sync()
        if warmup_ms > 0 and self.cuda:
            done = (time.perf_counter() - t0) * 1e3
            t1 = time.perf_counter()
            self.step()
            self.finish()
            self._sync()
            one = max((time.perf_counter() - t1) * 1e3, 1e-3)
            done += one
            extra = 0 if done >= warmup_ms else min(10_000, math.ceil((warmup_ms - done) / one))
            extra = int(reduce_scalar(self.ctx, float(extra), "max"))
            for _ in range(extra):
                self.step()
            self.finish()
            self._sync()
        return (time.perf_counter() - t0) * 1e3

    def timed(self, steps: int):
        """K steps bracketed by sync + barrier on both sides. Returns
        (max-over-ranks seconds, this rank's seconds, telemetry dict)."""
        self._sync()
        barrier(self.ctx)
        self._sync()
        self.recording = True
        with ClockSampler(self.ctx.device) as smp:
            t0 = time.perf_counter()
            for _ in range(steps):
                self.step()
            self.finish()
            issued = time.perf_counter() - t0  # host time to enqueue every step
            self._sync()
            barrier(self.ctx)
            self._sync()
            elapsed = time.perf_counter() - t0
        self.recording = False
        mine = elapsed
        if self.ctx.is_distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.ctx.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        tel = smp.result()
        tel["host_issue_ms"] = issued * 1e3
        return elapsed, mine, tel

    # -- the per-mode check -------------------------------------------------------
    def _last_slots(self, per_step: int):
        """Ring slots the most recent step wrote: the pipeline's last
        ``per_step`` units, or (serialized fallback) slots 0..per_step-1."""
        if self.pipe is not None:
            k = self.pipe.k
            return [u % self.pipe.R for u in range(max(k - per_step, 0), k)]
        return list(range(per_step))

    def verify(self) -> dict:
        """Check the data of one more step, run AFTER the timed region
        (parallel/verify.py; the reference's validate_result intent,
        matmul_scaling_benchmark.py:240-249, applied to every mode's output and
        collective). The A operands' signs are flipped first (exact in every
        dtype), so this step's products are the exact negation of every earlier
        step's: a collective that delivered a stale buffer — a peer's previous
        output, a ring slot not yet rewritten — is off by twice the value and
        fails. Per target of the step:

          * ``gemm``: 24 sampled rows of C against an fp32 recompute of A @ B;
          * ``reduce`` (batch_parallel): the same rows of the reduced C against
            the fp32 all-reduce (torch.distributed) of every rank's fp32
            recompute, and the reduced C's digest identical on every rank;
          * ``gather`` (matrix_parallel): every block of the gathered output
            bitwise equal (parallel/verify.py ``digest``) to its producer rank's
            local C.

        Collective (every rank runs the same targets). Returns ``{"check":
        "pass" | "fail" | "skipped", "check_detail": ...}``, agreed across ranks."""
        from pytorch_distributed_matmul_benchmark_amd.parallel.verify import (
            REL_TOL, digest, flip_sign_, ref_rows, rows_error, rows_of, sample_rows)

        ctx, ws = self.ctx, self.ctx.world_size
        if self.mode == "ring_parallel":
            return {"check": "skipped", "check_detail": "ring_parallel: no per-mode check"}
        for x in self._negate:
            flip_sign_(x)
        self.step()
        self.finish()
        self._sync()
        corrupt = self._test_corrupt_rank is not None and self._test_corrupt_rank == ctx.rank
        worst, fails = {}, []

        def note(key, err, tol):
            worst[key] = max(worst.get(key, 0.0), err)
            if not err <= tol:
                fails.append(f"{key} error {err:.3g} > {tol:.3g}")

        def gathered_digests(d: int):
            if not ctx.is_distributed:
                return [d]
            t = torch.tensor([d], dtype=torch.int64, device=ctx.device)
            out = torch.empty(ws, dtype=torch.int64, device=ctx.device)
            dist.all_gather_into_tensor(out, t)
            return [int(v) for v in out.tolist()]

        for kind, *ops in self._targets():
            if kind in ("gemm", "reduce"):
                A, B, C = ops
                if corrupt:
                    C.view(-1)[0] = 1e4  # row 0 is always sampled
                    corrupt = False
                rows = sample_rows(C.shape[0])
                pre = ref_rows(A, B, rows)
                tol = REL_TOL.get(C.dtype, 2.0 ** -6)
                if kind == "gemm":
                    note("gemm", rows_error(rows_of(C, rows), pre), tol)
                    continue
                both = torch.stack([pre, pre.abs()])
                if ctx.is_distributed:
                    dist.all_reduce(both)
                note("reduce", rows_error(rows_of(C, rows), both[0], both[1]), tol * (ws + 2) / 4)
                ds = gathered_digests(digest(C))
                if len(set(ds)) != 1:
                    fails.append("reduced output differs between ranks")
            else:  # gather
                local, gathered = ops
                if corrupt:
                    gathered.view(-1)[0] += 1
                    corrupt = False
                ds = gathered_digests(digest(local))
                rows = local.shape[0]
                bad = [j for j in range(ws) if digest(gathered[j * rows:(j + 1) * rows]) != ds[j]]
                worst["gather_blocks_wrong"] = worst.get("gather_blocks_wrong", 0) + len(bad)
                if bad:
                    fails.append(f"gathered blocks of ranks {bad} differ from their producers")
        ok = all_ok(ctx, not fails)
        detail = {k: (round(v, 6) if isinstance(v, float) else v) for k, v in worst.items()}
        if fails:
            detail["failed"] = fails[:4]
        elif not ok:
            detail["failed"] = ["on another rank"]
        return {"check": "pass" if ok else "fail", "check_detail": detail}

    def close(self):
        if self.pipe is not None:
            self.pipe.close()
        for fn in self._closers:  # IpcGather: unmap peers' buffers (collective barrier)
            if fn is not None:
                fn()
        self._closers = []


def _free(ctx) -> None:
    gc.collect()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)
        torch.cuda.empty_cache()


def _self_launch(a) -> int:
    """``--gpus N > 1`` outside torchrun: start N ranks as a child
    ``torch.distributed.run`` (the reference's launcher pattern,
    run_scaling_benchmark.sh:23-31) and exit with its code. Nothing here
    touches HIP (``import torch`` does not initialise it; the GPU count comes
    from sysfs / amdsmi, utils/telemetry.py), so the child ranks own their
    devices from scratch; the parent only waits."""
    import subprocess

    if a.device == "cuda" and a.dist_backend in ("auto", "nccl"):
        ndev = visible_gpus()
        if ndev < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but only {ndev} GPU(s) visible; RCCL needs one GPU "
                  f"per rank (use --dist-backend gloo to rehearse more ranks than GPUs)",
                  file=sys.stderr, flush=True)
            return 2
    # no --master-port: --standalone binds port 0 itself (a port picked here
    # could be taken by another process before the child listens on it)
    where = ([f"--master-addr=127.0.0.1", f"--master-port={a.master_port}"] if a.master_port
             else ["--standalone", "--local-addr=127.0.0.1"])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", *where, os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, PDMB_BENCH_CHILD="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


_T0 = time.perf_counter()


def _phase(ctx, key: str, phase: str) -> None:
    """Diagnostics (PDMB_BENCH_TRACE=1): each rank's mode / phase on stderr,
    with the seconds since start and this rank's peak device memory so far."""
    if os.environ.get("PDMB_BENCH_TRACE") == "1":
        mem = (f" peak {torch.cuda.max_memory_allocated(ctx.device) / 2**30:.2f} GiB"
               if ctx.device.type == "cuda" else "")
        print(f"[rank {ctx.rank} +{time.perf_counter() - _T0:.1f}s] {key}: {phase}{mem}",
              file=sys.stderr, flush=True)


def _fault(ctx, key: str, phase: str) -> None:
    """Fault injection for the failure-agreement tests: ``PDMB_BENCH_FAULT=
    rank:mode:phase`` (mode ``*`` = any; phase ``setup`` | ``timed``) raises
    on that rank at that point."""
    spec = os.environ.get("PDMB_BENCH_FAULT")
    if not spec:
        return
    r, m, p = spec.split(":")
    if int(r) == ctx.rank and m in (key, "*") and p == phase:
        raise RuntimeError(f"injected fault (rank {ctx.rank}, {key}, {phase})")


class _Pending:
    """Rank 0's JSON line from the moment the headline is measured. The
    secondary modes run after it and fill ``modes`` in place; if one of them
    takes the job down — a timed-region failure on rank 0 (``_die``) or
    torchrun's SIGTERM after another rank died or the driver's time limit — the
    line is still printed, with the modes that finished and ``modes_incomplete``
    saying why the rest did not, so a node run never loses its headline value.
    Printed at most once."""
    line = None
    lock = threading.Lock()

    @classmethod
    def emit(cls, why: str | None = None) -> bool:
        with cls.lock:
            out, cls.line = cls.line, None
        if out is None:
            return False
        if why:
            out["modes_incomplete"] = why
        sys.stdout.write(json.dumps(out) + "\n")
        sys.stdout.flush()
        return True


def _arm_pending_on_signals() -> None:
    """SIGTERM / SIGINT print the pending line, then exit 128 + signo. The work
    happens on a watcher thread woken through ``signal.set_wakeup_fd`` (written
    by the C-level handler at once): the main thread may be blocked inside a
    collective, where a Python-level handler would never get to run."""
    r, w = os.pipe()
    os.set_blocking(w, False)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda signo, frame: None)
    signal.set_wakeup_fd(w)

    def watch():
        while True:
            b = os.read(r, 1)
            if b and b[0] in (signal.SIGTERM, signal.SIGINT):
                _Pending.emit(f"terminated by signal {b[0]} during the secondary modes")
                os._exit(128 + b[0])
    threading.Thread(target=watch, daemon=True, name="pending-line").start()


def _die(ctx, key: str, exc: BaseException) -> None:
    """A failure inside a timed region cannot be agreed on (the other ranks are
    already blocked in a collective this rank will never join): report it and
    exit at once, so torchrun's agent tears the job down in seconds instead of
    every peer waiting out the process-group timeout."""
    import traceback

    print(f"[rank {ctx.rank}] {key} failed in the timed region: {exc!r}", file=sys.stderr,
          flush=True)
    traceback.print_exc(file=sys.stderr)
    sys.stderr.flush()
    if ctx.is_main:
        _Pending.emit(f"{key} failed in the timed region on rank 0: {exc!r}")
    sys.stdout.flush()
    os._exit(1)


def _measure(a, ctx, mode: str, overlap: bool, warmup: int, steps: int, key: str,
             warmup_ms: float = 0.0, batch: int = 1, test_corrupt_rank: int | None = None):
    """Build (agreed across ranks), time, then check (``Workload.verify``,
    outside the timed region) one workload. Returns ``(tflops, seconds,
    info)`` — ``info["check"]`` is "pass" / "fail" / "skipped" — or ``(None,
    None, error_string)``."""
    w, err = None, None
    _phase(ctx, key, "setup")
    try:
        _fault(ctx, key, "setup")
        w = Workload(a, ctx, mode, overlap, batch=batch, test_corrupt_rank=test_corrupt_rank)
    except Exception as e:  # OOM, unsupported shape, ...: every rank skips together
        err = f"{type(e).__name__}: {e}"
        print(f"[rank {ctx.rank}] {key} setup failed: {err}", file=sys.stderr, flush=True)
    if not all_ok(ctx, err is None):
        if w is not None:
            w.close()
        del w
        _free(ctx)
        return None, None, err or "failed on another rank"
    try:
        _fault(ctx, key, "timed")
        _phase(ctx, key, "warm")
        wms = w.warm(warmup, warmup_ms)
        _phase(ctx, key, "timed")
        el, mine, tel = w.timed(steps)
        _phase(ctx, key, "check")
        t_check = time.perf_counter()
        checked = w.verify()
        checked["check_s"] = round(time.perf_counter() - t_check, 3)
    except Exception as e:
        _die(ctx, key, e)
    _phase(ctx, key, "close")
    v = w.flops * steps / el / 1e12 if el > 0 else 0.0
    # per-rank rate: this rank's share of the FLOPs over its own wall time
    share = w.flops / ctx.world_size if mode in ("independent", "batch_parallel") else w.flops
    rates = gather_scalars(ctx, share * steps / mine / 1e12 if mine > 0 else 0.0)
    clocks = gather_scalars(ctx, tel["sclk_mhz"] or 0.0)
    comp, comm = w.split_ms()
    info = dict(global_batch=w.global_batch, parallelism=w.parallelism, kernel=w.kernel,
                warmup_ms=round(wms, 1),
                per_rank_tflops={"min": round(min(rates), 4), "max": round(max(rates), 4)},
                sclk_mhz=tel["sclk_mhz"], power_w=tel["power_w"],
                sclk_samples=tel["sclk_samples"], power_samples=tel["power_samples"],
                power_key=tel["power_key"],
                sclk_mhz_min_over_ranks=(round(min(clocks), 1) if min(clocks) > 0 else None),
                # host enqueue time per step (rank max) against ms_per_step: a host-bound
                # schedule shows host_issue close to the step time with the GPU waiting
                host_issue_ms_per_step=round(max(gather_scalars(ctx, tel["host_issue_ms"])) / steps, 4),
                **checked)
    if comp is not None:
        info["compute_ms"], info["comm_ms"] = round(comp, 4), round(comm, 4)
    if w.coll_choice is not None:
        info["collective"] = w.coll_choice
    if w._mask is not None:
        info["comm_cus"] = len(w._mask.excluded)   # --comm-cus rounded to 4 per XCD
    if w.plan is not None:
        info["plan"] = w.plan.as_dict()
        info["plan"]["signalled"] = bool(w.pipe is not None and w.pipe.signalled)
    w.close()
    del w
    _free(ctx)
    return v, el, info


def _rank0_alone(a, ctx, warmup: int, steps: int, warmup_ms: float, batch: int = 1):
    """TFLOPS of ``batch`` N x N GEMMs per step on rank 0 ALONE (the others wait
    at a barrier), measured inside this job: the '1 GPU' denominator of a
    scaling efficiency. The reference's own "Scaling efficiency" is rank
    imbalance, not scaling (matmul_scaling_benchmark.py:315)."""
    val = 0.0
    barrier(ctx)
    if ctx.rank == 0:
        try:
            one = DistContext(rank=0, world_size=1, local_rank=ctx.local_rank, device=ctx.device)
            w = Workload(a, one, "independent", False, batch=batch)
            w.warm(warmup, warmup_ms)
            el, _, _ = w.timed(steps)
            val = w.flops * steps / el / 1e12 if el > 0 else 0.0
            del w
        except Exception as e:  # a failed reference is "no efficiency", never a hang
            print(f"[rank 0] single-GPU reference failed: {e!r}", file=sys.stderr, flush=True)
            val = 0.0
        _free(ctx)
    barrier(ctx)
    v = reduce_scalar(ctx, val, "sum")
    return v if v > 0 else None


def _rccl_version(ctx):
    if not (ctx.is_distributed and ctx.backend == "nccl"):
        return None
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--dtype", default="bfloat16", choices=list(DTYPES))
    ap.add_argument("--mode", default="independent",
                    choices=["independent", "batch_parallel", "matrix_parallel", "ring_parallel"])
    ap.add_argument("--overlap", action="store_true",
                    help="batch/matrix_parallel: hide the collective behind the GEMMs")
    ap.add_argument("--chunks", type=int, default=0,
                    help="overlap: collective pieces per GEMM, each started by the GEMM's own "
                         "completion signals (0: the planner's choice; 1: whole collectives, "
                         "pipelined across GEMMs)")
    ap.add_argument("--comm-cus", type=int, default=0,
                    help="overlap: CUs kept free of GEMM workgroups for RCCL (CU-masked "
                         "compute stream; 0 = no mask)")
    ap.add_argument("--allreduce", default=None, choices=["rccl", "direct", "ipc", "auto"],
                    help="batch_parallel all-reduce: RCCL, a two-shot exchange over P2P links "
                         "(reduce-scatter group, native fp32 sum, all-gather group), the same "
                         "over xGMI peer memory (ipc), or auto: the fastest of the three, timed "
                         "on the job's ranks (default: rccl serialized, auto overlapped)")
    ap.add_argument("--allgather", default=None, choices=["rccl", "direct", "ipc", "auto"],
                    help="matrix_parallel all-gather: RCCL, direct P2P to every peer at once, "
                         "a pull over xGMI peer memory (ipc), or auto: the fastest, timed "
                         "(default: rccl serialized, auto overlapped)")
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: torch.matmul + gloo, to exercise the multi-rank path without a GPU")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--master-port", type=int, default=0,
                    help="self-launch rendezvous port (0: a free one)")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="timed steps for each secondary mode reported under \"modes\" "
                         "(batch_parallel / matrix_parallel, serialized and overlapped); 0: skip")
    ap.add_argument("--extra-warmup", type=int, default=3)
    ap.add_argument("--extra-warmup-ms", type=float, default=300.0,
                    help="secondary modes (and their rank-0 references) warm up for at least "
                         "this much wall time (GPU only)")
    ap.add_argument("--extra-deadline-s", type=float, default=240.0,
                    help="rank 0 prints its line (modes_incomplete) and ends the job if the "
                         "secondary modes run longer than this (0: no limit)")
    ap.add_argument("--no-scaling-ref", action="store_true",
                    help="skip the in-job rank-0-alone references (scaling_efficiency = null at N > 1)")
    return ap


def main() -> int:
    a = build_parser().parse_args()

    hooks = testhooks.active()
    if hooks:  # negative-control fault injection (racy collectives): never a measurement
        print(f"bench.py: refusing to run with test-only fault injection set: {', '.join(hooks)}",
              file=sys.stderr, flush=True)
        return 2
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            return _self_launch(a)
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}",
              file=sys.stderr, flush=True)
        return 2

    ctx = setup_distributed(a.device, timeout_s=float(os.environ.get("PDMB_PG_TIMEOUT", "300")),
                            backend=None if a.dist_backend == "auto" else a.dist_backend)
    cuda = ctx.device.type == "cuda"
    ws = ctx.world_size
    dt = DTYPES[a.dtype]
    headline16k = dt == torch.bfloat16 and a.size == 16384 and cuda
    # The collective self-test gates the job (matmul_scaling_benchmark.py:388-394).
    verified = verify_collectives(ctx, verbose=False) if ctx.is_distributed else None
    if verified is False:
        if ctx.is_main:
            print("bench.py: collective self-test failed", file=sys.stderr, flush=True)
        cleanup_distributed()
        return 1

    def vs_base(mode, value):
        base = BASELINE_TFLOPS.get(mode, {}).get(ws) if headline16k else None
        return round(value / base, 3) if base and value is not None else None

    # Headline: the metric BASELINE.json names, measured first on a quiet node.
    value, elapsed, head = _measure(a, ctx, a.mode, a.overlap, a.warmup, a.steps, a.mode)
    if value is None:
        if ctx.is_main:
            print(f"bench.py: headline {a.mode} failed: {head}", file=sys.stderr, flush=True)
        cleanup_distributed()
        return 1
    ms_step = elapsed / max(a.steps, 1) * 1e3

    single = value if ws == 1 and a.mode == "independent" else None
    if ws > 1 and not a.no_scaling_ref:
        single = _rank0_alone(a, ctx, a.warmup, a.steps, 0.0)

    def eff(v, ref):
        return round(v / (ws * ref), 4) if ref and v is not None else None

    modes = {}
    # a failed output check voids the number (Workload.verify: the step's data)
    head_ok = head.get("check") != "fail"
    if ctx.is_main:
        out = {
            "metric": METRIC, "value": round(value, 4) if head_ok else None, "unit": "TFLOPS",
            "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if a.mode in ("matrix_parallel", "ring_parallel") else "weak",
            "vs_baseline": vs_base(a.mode, value),
            "scaling_efficiency": eff(value, single),
            "single_gpu_tflops": round(single, 4) if single else None,
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32",
                      "float8_e4m3fn": "fp8_e4m3"}[a.dtype],
            "data": "synthetic (torch.randn N(0,1) operands, seeded per rank)",
            "device": ctx.device.type,
            "config": {"model": f"gemm_{a.size}x{a.size}x{a.size}_{a.dtype}",
                       "global_batch": head["global_batch"], "seq_len": a.size,
                       "parallelism": head["parallelism"], "mode": a.mode,
                       "overlap": bool(a.overlap), "backend": a.backend, "kernel": head["kernel"]},
            "dist_backend": ctx.backend,
            "collectives": {"all_reduce": a.allreduce or "rccl serialized, auto overlapped",
                            "all_gather": a.allgather or "rccl serialized, auto overlapped"},
            "world_size_seen": dist.get_world_size() if ctx.is_distributed else 1,
            "rccl_version": _rccl_version(ctx),
            "collectives_verified": verified,
            # the headline step's own output, checked after the timed region
            "check": head["check"], "check_detail": head["check_detail"], "check_s": head["check_s"],
            "per_rank_tflops": head["per_rank_tflops"],
            # medians of a 5 ms amdsmi poll over the timed region, with the sample counts
            "sclk_mhz": head["sclk_mhz"], "power_w": head["power_w"],
            "sclk_samples": head["sclk_samples"], "power_samples": head["power_samples"],
            "power_key": head["power_key"],
            "sclk_mhz_min_over_ranks": head["sclk_mhz_min_over_ranks"],
            "per_gpu_tflops": (round(value / ws, 2)
                               if a.mode not in ("matrix_parallel", "ring_parallel") else None),
            "vs_reference_1gpu_linear": round(value / (140.0 * ws), 3),
            "modes": modes,
        }
        if "plan" in head:
            out["config"]["overlap_plan"] = head["plan"]
        _Pending.line = out
        _arm_pending_on_signals()

    # Secondary modes (BASELINE configs 4-5), each family after its own
    # rank-0-alone reference of the same per-rank shape. At ws = 1 there is no
    # collective to overlap: those entries are null.
    if a.extra_steps > 0 and ctx.is_main and a.extra_deadline_s > 0:
        # a secondary mode stuck in a collective (a peer lost, a hang) must not
        # outlive the process-group timeout with the headline unprinted
        def deadline():
            time.sleep(a.extra_deadline_s)
            if _Pending.emit(f"secondary modes still running after {a.extra_deadline_s:g} s"):
                os._exit(3)
        threading.Thread(target=deadline, daemon=True, name="extra-deadline").start()
    if a.extra_steps > 0:
        wms = a.extra_warmup_ms
        for family, ref_batch in (("batch_parallel", local_batch(ws)), ("matrix_parallel", 1)):
            ref = None
            if not a.no_scaling_ref or ws == 1:
                ref = _rank0_alone(a, ctx, a.extra_warmup, a.extra_steps, wms, batch=ref_batch)
            for ov in (False, True):
                if family == a.mode and ov == a.overlap:
                    continue
                key = family + ("+overlap" if ov else "")
                if ov and ws == 1:
                    modes[key] = None
                    continue
                v, el, info = _measure(a, ctx, family, ov, a.extra_warmup, a.extra_steps, key,
                                       warmup_ms=wms)
                if v is None:
                    modes[key] = {"error": info}
                    continue
                if info.get("check") == "fail":  # checked wrong: no number for this mode
                    v = None
                modes[key] = {"value": round(v, 4) if v is not None else None,
                              "ms_per_step": round(el / a.extra_steps * 1e3, 4),
                              "steps": a.extra_steps, "warmup": a.extra_warmup,
                              "scaling": "strong" if family == "matrix_parallel" else "weak",
                              "vs_baseline": vs_base(family, v),
                              "scaling_efficiency": eff(v, ref) if v is not None else None,
                              "ref_tflops_rank0_alone": round(ref, 4) if ref else None, **info}

    _Pending.emit()
    cleanup_distributed()
    return 0 if head_ok else 1


if __name__ == "__main__":
    sys.exit(main())
