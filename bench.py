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
comm stream — for ``--extra-steps`` steps each, and reports them under
``"modes"`` in the same JSON line, so one launch at N GPUs yields the
BASELINE configs 3-5 (``--extra-steps 0`` skips them).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.comm import (CommStream,  # noqa: E402
                                                                   new_event)
from pytorch_distributed_matmul_benchmark_amd.parallel.dist import (  # noqa: E402
    barrier, cleanup_distributed, setup_distributed)
from pytorch_distributed_matmul_benchmark_amd.parallel.partition import (  # noqa: E402
    column_shard, effective_chunks, global_batch, local_batch, row_chunks)

# Reference numbers (README.md:43-46): whole-system TFLOPS at 16k bf16.
BASELINE_TFLOPS = {"independent": {1: 140.0, 2: 294.0},
                   "batch_parallel": {1: 140.0, 2: 237.0},
                   "matrix_parallel": {1: 140.0, 2: 141.0}}
METRIC = "TFLOPS (whole node) + scaling efficiency, 16k×16k bf16 GEMM at 1/2/4/8 GPUs"
DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
          "float8_e4m3fn": torch.float8_e4m3fn}


class Workload:
    """Operands + one timed ``step()`` of a scaling mode on this rank."""

    def __init__(self, a, ctx, mode: str, overlap: bool):
        self.ctx, self.mode, self.overlap = ctx, mode, overlap
        self.cuda = ctx.device.type == "cuda"
        self.dt = DTYPES[a.dtype]
        self.backend = a.backend
        dev, n, ws, dt = ctx.device, a.size, ctx.world_size, self.dt
        odt = gemm.out_dtype(dt)  # fp8 operands write a bf16 C
        self._g = torch.Generator(device=dev)
        flop_gemm = 2.0 * n * n * n
        comp = torch.cuda.current_stream(dev) if self.cuda else None
        overlap = overlap and ws > 1

        if mode == "independent":
            A, B = self._rnd(n, n, seed=2 * ctx.rank), self._rnd(n, n, seed=2 * ctx.rank + 1, b=True)
            C = torch.empty(n, n, device=dev, dtype=odt)
            self.kernel = self._label(A, B, C)

            def step():
                self._mm(A, B, C)
            self.flops = flop_gemm * ws
            self.global_batch, self.parallelism = ws, f"independent{ws}"
        elif mode == "batch_parallel":
            lb, gb = local_batch(ws), global_batch(ws)
            A = self._rnd(lb, n, n, seed=2 * ctx.rank)
            B = self._rnd(lb, n, n, seed=2 * ctx.rank + 1, b=True)
            C = torch.empty(lb, n, n, device=dev, dtype=odt)
            self.kernel = self._label(A, B, C)
            if overlap:
                cs = CommStream(dev)
                ch = effective_chunks(n, n, a.chunks) if self.cuda else a.chunks
                units = [(b, s, e) for b in range(lb) for (s, e) in row_chunks(n, ch)]
                ready = [new_event(dev) for _ in units]
                done = [new_event(dev) for _ in units]

                def step():
                    for u, (b, s, e) in enumerate(units):
                        if self.cuda:
                            comp.wait_event(done[u])
                        self._mm(A[b, s:e], B[b], C[b, s:e])
                        ready[u].record(comp)
                        cs.all_reduce(C[b, s:e], after=ready[u], done=done[u])
                    if self.cuda:
                        for d in done:
                            comp.wait_event(d)
            else:
                def step():
                    self._mm(A, B, C)
                    if ws > 1:
                        dist.all_reduce(C)
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
            Cl = torch.empty(n, sh.padded, device=dev, dtype=odt)
            self.kernel = self._label(A, Bl, Cl)
            if overlap:
                cs = CommStream(dev)
                rc = row_chunks(n, effective_chunks(n, sh.padded, a.chunks) if self.cuda
                                else a.chunks)
                bufs = [torch.empty(ws * (e - s), sh.padded, device=dev, dtype=odt) for s, e in rc]
                ready = [new_event(dev) for _ in rc]
                done = [new_event(dev) for _ in rc]

                def step():
                    for j, (s, e) in enumerate(rc):
                        if self.cuda:
                            comp.wait_event(done[j])
                        self._mm(A[s:e], Bl, Cl[s:e])
                        ready[j].record(comp)
                        cs.all_gather_into(bufs[j], Cl[s:e], after=ready[j], done=done[j])
                    if self.cuda:
                        for d in done:
                            comp.wait_event(d)
            else:
                gathered = torch.empty(ws * n, sh.padded, device=dev, dtype=odt)

                def step():
                    self._mm(A, Bl, Cl)
                    if ws > 1:
                        dist.all_gather_into_tensor(gathered, Cl)
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"tp{ws}"
        elif mode == "ring_parallel":
            # Opt-in (not timed by default): all-gather-GEMM over the ring,
            # models/ring_parallel.py. A row blocks rotate by P2P behind each hop's GEMM.
            rs, sh = column_shard(n, ws, ctx.rank, align=256), column_shard(n, ws, ctx.rank, align=8)
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
            R = [torch.empty_like(Al), torch.empty_like(Al)]
            self.kernel = self._label(Al, Bl, Cl[:rp])
            cs = CommStream(dev)
            gdone = [new_event(dev) for _ in range(ws)]
            rdone = [new_event(dev) for _ in range(max(ws - 1, 0))]
            last = [None]
            nxt, prv = (ctx.rank + 1) % ws, (ctx.rank - 1) % ws

            def step():
                cur = Al
                for s in range(ws):
                    if s > 0 and self.cuda:
                        comp.wait_event(rdone[s - 1])
                    if s < ws - 1:
                        cs.exchange(cur, nxt, R[(s + 1) % 2], prv, after=last[0], done=rdone[s])
                    j = (ctx.rank - s) % ws
                    self._mm(cur, Bl, Cl[j * rp:(j + 1) * rp])
                    gdone[s].record(comp)
                    last[0] = gdone[s]
                    if s < ws - 1:
                        cur = R[(s + 1) % 2]
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"ring{ws}"
        else:
            raise ValueError(mode)
        self.step = step

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
            return torch._scaled_mm(A, B, scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                    out=out)
        if (self.backend == "torch" or not self.cuda) and self.dt != gemm.FP8:
            return torch.matmul(A, B, out=out)
        return gemm.matmul(A, B, out=out)

    def _label(self, A, B, C):
        if not self.cuda:
            return "torch.matmul(cpu)"
        return gemm.kernel_for(A, B, C) if self.backend == "native" else "hipBLASLt"

    def _sync(self):
        if self.cuda:
            torch.cuda.synchronize(self.ctx.device)

    def timed(self, warmup: int, steps: int) -> float:
        """W untimed steps, then K steps bracketed by sync+barrier; max-over-ranks seconds."""
        for _ in range(warmup):
            self.step()
        self._sync()
        barrier(self.ctx)
        self._sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        self._sync()
        barrier(self.ctx)
        self._sync()
        elapsed = time.perf_counter() - t0
        if self.ctx.is_distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.ctx.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed


def _free(ctx) -> None:
    gc.collect()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)
        torch.cuda.empty_cache()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--dtype", default="bfloat16", choices=list(DTYPES))
    ap.add_argument("--mode", default="independent",
                    choices=["independent", "batch_parallel", "matrix_parallel", "ring_parallel"])
    ap.add_argument("--overlap", action="store_true",
                    help="batch/matrix_parallel: hide the collective behind the GEMM chunks")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: torch.matmul + gloo, to exercise the multi-rank path without a GPU")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="timed steps for each secondary mode reported under \"modes\" "
                         "(batch_parallel / matrix_parallel, serialized and overlapped); 0: skip")
    ap.add_argument("--extra-warmup", type=int, default=3)
    a = ap.parse_args()

    ctx = setup_distributed(a.device, backend=None if a.dist_backend == "auto" else a.dist_backend)
    cuda = ctx.device.type == "cuda"
    ws = ctx.world_size
    if ws != a.gpus and ctx.is_main:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={ws}; using {ws}", file=sys.stderr)
    dt = DTYPES[a.dtype]
    headline16k = dt == torch.bfloat16 and a.size == 16384 and cuda

    def vs_base(mode, value):
        base = BASELINE_TFLOPS.get(mode, {}).get(ws) if headline16k else None
        return round(value / base, 3) if base else None

    # Headline: the metric BASELINE.json names, measured first on a quiet node.
    w = Workload(a, ctx, a.mode, a.overlap)
    elapsed = w.timed(a.warmup, a.steps)
    ms_step = elapsed / max(a.steps, 1) * 1e3
    value = w.flops * a.steps / elapsed / 1e12 if elapsed > 0 else 0.0
    head = dict(global_batch=w.global_batch, parallelism=w.parallelism, kernel=w.kernel)
    del w
    _free(ctx)

    # Secondary modes (BASELINE configs 4-5): same operands' shapes and dtype, own timing.
    modes = {}
    if a.extra_steps > 0:
        for mode, ov in (("batch_parallel", False), ("batch_parallel", True),
                         ("matrix_parallel", False), ("matrix_parallel", True)):
            if mode == a.mode and ov == a.overlap:
                continue
            key = mode + ("+overlap" if ov else "")
            w = Workload(a, ctx, mode, ov)
            el = w.timed(a.extra_warmup, a.extra_steps)
            v = w.flops * a.extra_steps / el / 1e12 if el > 0 else 0.0
            modes[key] = {"value": round(v, 4), "ms_per_step": round(el / a.extra_steps * 1e3, 4),
                          "steps": a.extra_steps, "warmup": a.extra_warmup,
                          "global_batch": w.global_batch, "parallelism": w.parallelism,
                          "scaling": "strong" if mode == "matrix_parallel" else "weak",
                          "vs_baseline": vs_base(mode, v), "kernel": w.kernel}
            del w
            _free(ctx)

    if ctx.is_main:
        out = {
            "metric": METRIC, "value": round(value, 4), "unit": "TFLOPS",
            "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if a.mode in ("matrix_parallel", "ring_parallel") else "weak",
            "vs_baseline": vs_base(a.mode, value),
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32",
                      "float8_e4m3fn": "fp8_e4m3"}[a.dtype],
            "data": "synthetic (torch.randn N(0,1) operands, seeded per rank)",
            "device": ctx.device.type,
            "config": {"model": f"gemm_{a.size}x{a.size}x{a.size}_{a.dtype}",
                       "global_batch": head["global_batch"], "seq_len": a.size,
                       "parallelism": head["parallelism"], "mode": a.mode,
                       "overlap": bool(a.overlap), "backend": a.backend, "kernel": head["kernel"]},
            "per_gpu_tflops": (round(value / ws, 2)
                               if a.mode not in ("matrix_parallel", "ring_parallel") else None),
            "vs_reference_1gpu_linear": round(value / (140.0 * ws), 3),
            "modes": modes,
        }
        print(json.dumps(out), flush=True)
    cleanup_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
