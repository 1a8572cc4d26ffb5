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

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
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


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16", "float32"])
    ap.add_argument("--mode", default="independent",
                    choices=["independent", "batch_parallel", "matrix_parallel"])
    ap.add_argument("--overlap", action="store_true",
                    help="batch/matrix_parallel: hide the collective behind the GEMM chunks")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: torch.matmul + gloo, to exercise the multi-rank path without a GPU")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    a = ap.parse_args()

    ctx = setup_distributed(a.device, backend=None if a.dist_backend == "auto" else a.dist_backend)
    cuda = ctx.device.type == "cuda"
    ws = ctx.world_size
    if ws != a.gpus and ctx.is_main:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={ws}; using {ws}", file=sys.stderr)
    dt = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}[a.dtype]
    dev, n = ctx.device, a.size
    g = torch.Generator(device=dev)

    def rnd(*shape, seed):
        g.manual_seed(seed)
        return torch.randn(*shape, generator=g, device=dev, dtype=dt)

    def mm(A, B, out):
        if a.backend == "torch" or not cuda:
            return torch.matmul(A, B, out=out)
        return gemm.matmul(A, B, out=out)

    def label(A, B, C):
        if not cuda:
            return "torch.matmul(cpu)"
        return gemm.kernel_for(A, B, C) if a.backend == "native" else "hipBLASLt"

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    flop_gemm = 2.0 * n * n * n
    if a.mode == "independent":
        A, B = rnd(n, n, seed=2 * ctx.rank), rnd(n, n, seed=2 * ctx.rank + 1)
        C = torch.empty(n, n, device=dev, dtype=dt)
        kernel = label(A, B, C)

        def step():
            mm(A, B, C)
        flops_step = flop_gemm * ws
        cfg = dict(global_batch=ws, parallelism=f"independent{ws}")
    elif a.mode == "batch_parallel":
        lb, gb = local_batch(ws), global_batch(ws)
        A, B = rnd(lb, n, n, seed=2 * ctx.rank), rnd(lb, n, n, seed=2 * ctx.rank + 1)
        C = torch.empty(lb, n, n, device=dev, dtype=dt)
        kernel = label(A, B, C)
        comp = torch.cuda.current_stream(dev) if cuda else None
        if a.overlap and ws > 1:
            cs = CommStream(dev)
            ch = effective_chunks(n, n, a.chunks) if cuda else a.chunks
            units = [(b, s, e) for b in range(lb) for (s, e) in row_chunks(n, ch)]
            ready = [new_event(dev) for _ in units]
            done = [new_event(dev) for _ in units]

            def step():
                for u, (b, s, e) in enumerate(units):
                    if cuda:
                        comp.wait_event(done[u])
                    mm(A[b, s:e], B[b], C[b, s:e])
                    ready[u].record(comp)
                    cs.all_reduce(C[b, s:e], after=ready[u], done=done[u])
                if cuda:
                    for d in done:
                        comp.wait_event(d)
        else:
            def step():
                mm(A, B, C)
                if ws > 1:
                    dist.all_reduce(C)
        flops_step = flop_gemm * gb
        cfg = dict(global_batch=gb, parallelism=f"dp{ws}")
    else:
        sh = column_shard(n, ws, ctx.rank, align=8)
        A = rnd(n, n, seed=10_000)
        Bg = rnd(n, n, seed=10_001)
        Bl = torch.zeros(n, sh.padded, device=dev, dtype=dt)
        Bl[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
        del Bg
        Cl = torch.empty(n, sh.padded, device=dev, dtype=dt)
        gathered = torch.empty(ws * n, sh.padded, device=dev, dtype=dt)
        kernel = label(A, Bl, Cl)
        comp = torch.cuda.current_stream(dev) if cuda else None
        if a.overlap and ws > 1:
            cs = CommStream(dev)
            rc = row_chunks(n, effective_chunks(n, sh.padded, a.chunks) if cuda else a.chunks)
            bufs = [torch.empty(ws * (e - s), sh.padded, device=dev, dtype=dt) for s, e in rc]
            ready = [new_event(dev) for _ in rc]
            done = [new_event(dev) for _ in rc]

            def step():
                for j, (s, e) in enumerate(rc):
                    if cuda:
                        comp.wait_event(done[j])
                    mm(A[s:e], Bl, Cl[s:e])
                    ready[j].record(comp)
                    cs.all_gather_into(bufs[j], Cl[s:e], after=ready[j], done=done[j])
                if cuda:
                    for d in done:
                        comp.wait_event(d)
        else:
            def step():
                mm(A, Bl, Cl)
                if ws > 1:
                    dist.all_gather_into_tensor(gathered, Cl)
        flops_step = flop_gemm
        cfg = dict(global_batch=1, parallelism=f"tp{ws}")

    for _ in range(a.warmup):
        step()
    sync()
    barrier(ctx)
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    barrier(ctx)
    sync()
    elapsed = time.perf_counter() - t0
    if ctx.is_distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / max(a.steps, 1) * 1e3
    value = flops_step * a.steps / elapsed / 1e12 if elapsed > 0 else 0.0
    base = (BASELINE_TFLOPS[a.mode].get(ws)
            if dt == torch.bfloat16 and n == 16384 and cuda else None)
    if ctx.is_main:
        out = {
            "metric": METRIC, "value": round(value, 4), "unit": "TFLOPS",
            "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if a.mode == "matrix_parallel" else "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32"}[a.dtype],
            "data": "synthetic (torch.randn N(0,1) operands, seeded per rank)",
            "device": ctx.device.type,
            "config": {"model": f"gemm_{n}x{n}x{n}_{a.dtype}", "global_batch": cfg["global_batch"],
                       "seq_len": n, "parallelism": cfg["parallelism"], "mode": a.mode,
                       "overlap": bool(a.overlap), "backend": a.backend, "kernel": kernel},
            "per_gpu_tflops": round(value / ws, 2) if a.mode != "matrix_parallel" else None,
            "vs_reference_1gpu_linear": round(value / (140.0 * ws), 3),
        }
        print(json.dumps(out), flush=True)
    cleanup_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
