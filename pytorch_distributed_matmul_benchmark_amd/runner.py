"""The per-size benchmark driver behind every CLI entry point.

One implementation of the reference's four copy-pasted ``run_benchmarks`` /
``main`` pairs (SURVEY §1 "no shared module"):

  kind          entry point                               reference
  ----------    ---------------------------------------   -------------------------------------------
  basic         matmul_benchmark.py                       matmul_benchmark.py:81-200
  scaling       matmul_scaling_benchmark.py               matmul_scaling_benchmark.py:251-404
  distributed   backup/matmul_distributed_benchmark.py    backup/matmul_distributed_benchmark.py:176-319
  overlap       backup/matmul_overlap_benchmark.py        backup/matmul_overlap_benchmark.py:280-414

Same flags and defaults (``--sizes 4096 8192 16384 --iterations 50
--warmup 10 --dtype bfloat16 [--mode …]``), same rank-0 lines, plus opt-in
MI355X flags: ``--device``, ``--batch``, ``--overlap``, ``--chunks``,
``--graph``, ``--backend``, ``--kernel``, ``--check``, ``--json``,
``--single-gpu-tflops``.

Per size, every rank: run the mode → agree on success (error-flag
all-reduce) → reduce metrics → rank 0 prints and records.
"""
from __future__ import annotations

import argparse
import traceback
from typing import Dict, List, Optional

import torch

from .models import (DISTRIBUTED_MODES, EXTRA_SCALING_MODES, OVERLAP_MODES, SCALING_MODES,
                     ModeResult, Workload, run_mode)
from .models.common import tolerance
from .ops.gemm import KERNELS as _GEMM_KERNELS, out_dtype as _gemm_out_dtype
from .parallel.dist import (DistContext, all_ok, barrier, cleanup_distributed, reduce_scalar,
                            setup_distributed, verify_collectives)
from .utils.metrics import (balance_efficiency, bytes_per_element, dtype_from_name, dtype_name,
                            overlap_efficiency, peak_for_device, percent_of_peak,
                            scaling_efficiency, square_flops, tflops_from)
from .utils.report import Reporter, device_banner
from .utils import testhooks
from .utils.timing import marker

KINDS = {
    "basic": dict(title="Matrix Multiplication Benchmark", width=60, modes=("independent",),
                  default_mode="independent",
                  desc="Distributed PyTorch Matrix Multiplication Benchmark (MI355X)"),
    "scaling": dict(title="Matrix Multiplication Scaling Benchmark", width=70,
                    modes=SCALING_MODES + EXTRA_SCALING_MODES, default_mode="independent",
                    desc="Matrix Multiplication Scaling Benchmark (MI355X)"),
    "distributed": dict(title="Distributed Matrix Multiplication Benchmark", width=70,
                        modes=DISTRIBUTED_MODES, default_mode="data_parallel",
                        desc="Distributed Matrix Multiplication Benchmark with Communication"),
    "overlap": dict(title="Overlapped Communication/Computation Benchmark", width=70,
                    modes=OVERLAP_MODES, default_mode="overlap",
                    desc="Overlapped Communication/Computation Benchmark"),
}


def build_parser(kind: str) -> argparse.ArgumentParser:
    k = KINDS[kind]
    p = argparse.ArgumentParser(description=k["desc"])
    p.add_argument("--sizes", type=int, nargs="+", default=[4096, 8192, 16384],
                   help="Matrix sizes to benchmark (default: 4096 8192 16384)")
    p.add_argument("--iterations", type=int, default=50,
                   help="Number of iterations per benchmark (default: 50)")
    p.add_argument("--warmup", type=int, default=10,
                   help="Number of warmup iterations (default: 10)")
    p.add_argument("--dtype", type=str, default="bfloat16",
                   choices=["float32", "float16", "bfloat16", "float8_e4m3fn"],
                   help="Data type for matrices (default: bfloat16; float8_e4m3fn: OCP e4m3 "
                        "operands, bf16 output, on gfx950's block-scaled fp8 MFMA)")
    if kind != "basic":
        p.add_argument("--mode", type=str, default=k["default_mode"], choices=list(k["modes"]),
                       help=f"Benchmark mode (default: {k['default_mode']})")
    g = p.add_argument_group("MI355X options")
    g.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                   help="auto: this rank's GPU if present, else CPU (torch.matmul reference path)")
    g.add_argument("--backend", default="native", choices=["native", "torch"],
                   help="GEMM implementation on GPU: native gfx950 MFMA kernels (default) or "
                        "torch.matmul/hipBLASLt for A/B comparison")
    g.add_argument("--kernel", default="auto", choices=list(_GEMM_KERNELS),
                   help="native kernel selection (shipping kernels; A/B kernels need a "
                        "PDMB_EXPERIMENTS=1 build and scripts/ab_kernels.py)")
    g.add_argument("--batch", type=int, default=4,
                   help="batch_parallel global batch (rounded up to a multiple of the world size)")
    g.add_argument("--overlap", action="store_true",
                   help="batch/matrix_parallel: overlap the collective with the GEMM on a second stream")
    g.add_argument("--chunks", type=int, default=0,
                   help="--overlap: collective pieces per GEMM, each started by the GEMM's own "
                        "tile-completion signals (0: the overlap planner's choice; 1: whole "
                        "collectives pipelined across GEMMs)")
    g.add_argument("--allgather", default="rccl", choices=["rccl", "direct", "ipc", "auto"],
                   help="matrix_parallel all-gather: RCCL's all_gather_into_tensor; direct: one "
                        "batched P2P group sending this rank's shard to every peer at once (each "
                        "over its own xGMI link on a fully connected node); ipc: every rank pulls "
                        "the peers' shards out of their memory (hipIpc mappings) in one kernel "
                        "launch (CPU tensors: as direct); auto: the fastest of the three, timed on "
                        "the job's own ranks")
    g.add_argument("--allreduce", default="rccl", choices=["rccl", "direct", "ipc", "auto"],
                   help="batch_parallel / data_parallel / overlap all-reduce: RCCL's all_reduce; "
                        "direct: a two-shot exchange over point-to-point links (reduce-scatter as one "
                        "batched P2P group, native fp32-accumulating sum, all-gather as another); "
                        "ipc (GPUs): the same two shots read out of the peers' memory (hipIpc "
                        "mappings; the sum reads every peer's chunk in place); elsewhere as direct; "
                        "auto (batch_parallel): the fastest of the three, timed on the job's ranks "
                        "(other modes: rccl)")
    g.add_argument("--comm-cus", type=int, default=0,
                   help="--overlap: CUs kept free of GEMM workgroups for RCCL (CU-masked "
                        "compute stream, spread over the 8 XCDs; 0 = no mask)")
    g.add_argument("--graph", action="store_true",
                   help="independent: replay the timed loop as one hipGraph")
    g.add_argument("--check", action="store_true",
                   help="verify results against a float64 reference (sampled rows)")
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--min-warmup-ms", type=float, default=100.0,
                   help="extend the --warmup iterations until this much GPU time has run "
                        "(MI355X clocks settle under sustained MFMA load; 0 = exactly --warmup)")
    g.add_argument("--json", default=None, help="append one JSON record per result to this file")
    g.add_argument("--single-gpu-tflops", type=float, default=None,
                   help="measured 1-GPU TFLOPS for the 'efficiency vs 1 GPU' line")
    g.add_argument("--scaling-ref", action="store_true",
                   help="before each size, time the N×N GEMM on rank 0 ALONE (other ranks idle) "
                        "and report scaling efficiency = node TFLOPS / (ws × that)")
    g.add_argument("--timeout", type=float, default=600.0, help="process-group timeout (s)")
    g.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="auto: nccl (= RCCL) for GPU tensors, gloo for CPU; gloo on GPU tensors "
                        "lets several ranks share one GPU to rehearse the multi-rank paths")
    g.add_argument("--debug", action="store_true", help="print tracebacks of failed sizes")
    g.add_argument("--profile", action="store_true",
                   help="wrap each size in a roctx range (rocprofv3 --marker-trace --kernel-trace)")
    g.add_argument("--show-topology", action="store_true",
                   help="rank 0 prints the GPU interconnect (rocm-smi --showtopotype --showtopohops)")
    g.add_argument("--resume", action="store_true",
                   help="with --json: skip sizes whose (script, mode, dtype, ws) record already exists")
    return p


def _mode_of(kind: str, args) -> str:
    return getattr(args, "mode", None) or KINDS[kind]["default_mode"]


def _workload(args, n: int, dtype: torch.dtype) -> Workload:
    return Workload(n=n, dtype=dtype, iters=args.iterations, warmup=args.warmup, seed=args.seed,
                    backend=args.backend, kernel=args.kernel, batch=args.batch,
                    overlap=args.overlap, chunks=args.chunks,
                    comm_cus=args.comm_cus, allgather=args.allgather, allreduce=args.allreduce, graph=args.graph,
                    check=args.check,
                    min_warmup_ms=args.min_warmup_ms)


def _single_gpu_reference(ctx: DistContext, args, n: int, dtype: torch.dtype) -> float:
    """TFLOPS of one N×N GEMM on rank 0 while every other rank idles at a barrier:
    the '1 GPU' denominator of the scaling efficiency, measured in the same job
    on the same device and data distribution (broadcast to all ranks)."""
    from .models import independent

    val = 0.0
    barrier(ctx)
    if ctx.rank == 0:
        try:  # never skip the collectives below: a failure here becomes "no reference"
            w = _workload(args, n, dtype)
            w.iters, w.warmup, w.check = max(3, min(args.iterations, 10)), max(1, min(args.warmup, 3)), False
            one = DistContext(rank=0, world_size=1, local_rank=ctx.local_rank, device=ctx.device)
            val = independent.run(w, one).tflops
        except Exception as e:  # pragma: no cover
            print(f"[rank 0] single-GPU reference failed: {e!r}", flush=True)
            val = 0.0
    barrier(ctx)
    v = reduce_scalar(ctx, val, "sum")
    return v if v > 0 else None


def _aggregate(ctx: DistContext, r: ModeResult) -> Dict[str, Optional[float]]:
    """Cross-rank reductions (collective: every rank calls this in the same order)."""
    agg: Dict[str, Optional[float]] = {}
    agg["avg_ms"] = reduce_scalar(ctx, r.avg_ms, "avg")
    agg["max_ms"] = reduce_scalar(ctx, r.avg_ms, "max")
    agg["tflops_sum"] = reduce_scalar(ctx, r.tflops, "sum")
    agg["tflops_avg"] = reduce_scalar(ctx, r.tflops, "avg")
    agg["compute_ms"] = reduce_scalar(ctx, r.compute_ms or 0.0, "avg")
    agg["comm_ms"] = reduce_scalar(ctx, r.comm_ms or 0.0, "avg")
    agg["compute_only_tflops"] = reduce_scalar(ctx, r.compute_only_tflops or 0.0, "avg")
    agg["relerr"] = reduce_scalar(ctx, r.relerr if r.relerr is not None else -1.0, "max")
    if agg["relerr"] is not None and agg["relerr"] < 0:
        agg["relerr"] = None
    # Whole-node throughput: all FLOPs executed in one iteration ÷ slowest rank's time.
    agg["node_tflops"] = tflops_from(r.flops_total, agg["max_ms"] / 1e3)
    return agg


def _peak(ctx: DistContext):
    if not ctx.is_cuda:
        return None
    p = torch.cuda.get_device_properties(ctx.device)
    return peak_for_device(torch.cuda.get_device_name(ctx.device), getattr(p, "gcnArchName", ""))


def _print_results(kind: str, mode: str, rep: Reporter, ctx: DistContext, n: int,
                   dtype: torch.dtype, r: ModeResult, agg: Dict, args) -> Dict:
    ws = ctx.world_size
    extra: Dict[str, object] = {}
    rep.line(f"\nResults for {n}x{n}:")
    peak = _peak(ctx)
    if kind == "basic":
        rep.line(f"  - Average time per multiplication: {agg['avg_ms']:.3f} ms")
        rep.line(f"  - TFLOPS per GPU: {r.tflops:.2f}")
        rep.line(f"  - Total TFLOPS (all GPUs): {agg['tflops_sum']:.2f}")
        rep.line(f"  - Required FLOPs per operation: {square_flops(n) / 1e12:.2f} TFLOPs")
        pct = percent_of_peak(r.tflops, peak, dtype)
        if pct is not None:
            rep.line(f"  - GPU Efficiency: {pct:.1f}% of {peak.gpu} theoretical peak "
                     f"({peak.for_dtype(dtype):.1f} TFLOPS dense)")
    elif kind == "scaling":
        rep.line(f"  - Average time per operation: {agg['avg_ms']:.3f} ms")
        if mode == "independent":
            rep.line(f"  - TFLOPS per GPU: {r.tflops:.2f}")
            rep.line(f"  - Total system TFLOPS: {agg['tflops_sum']:.2f}")
            bal = balance_efficiency(agg["tflops_sum"], r.tflops, ws)
            rep.line(f"  - Scaling efficiency: {bal:.1f}% (rank balance: sum / (ws x rank 0))")
        elif mode == "batch_parallel":
            lb = r.extra.get("local_batch")
            gb = r.extra.get("global_batch")
            rep.line(f"  - Compute time: {agg['compute_ms']:.3f} ms, Comm time: {agg['comm_ms']:.3f} ms"
                     + (" (overlapped; comm = exposed part)" if r.extra.get("overlap") else ""))
            rep.line(f"  - TFLOPS per GPU: {r.tflops:.2f}")
            rep.line(f"  - Total system TFLOPS: {r.tflops * ws:.2f}")
            rep.line(f"  - Processing {gb} total batches across {ws} GPU(s) ({lb} per GPU)")
        else:
            rep.line(f"  - Compute time: {agg['compute_ms']:.3f} ms, Comm time: {agg['comm_ms']:.3f} ms"
                     + (" (overlapped; comm = exposed part)" if r.extra.get("overlap") else ""))
            rep.line(f"  - TFLOPS per GPU (portion): {r.tflops:.2f}")
            rep.line(f"  - Effective system TFLOPS: {agg['tflops_avg']:.2f}")
            rep.line(f"  - Each GPU processes 1/{ws} of the matrix")
        total_flops = {"independent": square_flops(n, ws),
                       "batch_parallel": square_flops(n, r.extra.get("global_batch", 4)),
                       "matrix_parallel": square_flops(n),
                       "ring_parallel": square_flops(n)}[mode]
        actual = tflops_from(total_flops, agg["avg_ms"] / 1e3)
        extra["actual_tflops"] = actual
        rep.line(f"  - Actual TFLOPS (total FLOPs / time): {actual:.2f}")
    elif kind == "distributed":
        rep.line(f"  - Total time per operation: {agg['avg_ms']:.3f} ms")
        if mode != "independent" and ws > 1:
            rep.line(f"  - Compute time: {agg['compute_ms']:.3f} ms")
            rep.line(f"  - Communication time: {agg['comm_ms']:.3f} ms")
            ov = 100.0 * agg["comm_ms"] / agg["avg_ms"] if agg["avg_ms"] > 0 else 0.0
            rep.line(f"  - Communication overhead: {ov:.1f}%")
        if mode == "independent":
            rep.line(f"  - TFLOPS per GPU: {r.tflops:.2f}")
            rep.line(f"  - Total TFLOPS (all GPUs): {agg['tflops_sum']:.2f}")
        else:
            rep.line(f"  - Effective TFLOPS: {agg['tflops_avg']:.2f}")
        rep.line(f"  - Required FLOPs per operation: {square_flops(n) / 1e12:.2f} TFLOPs")
        if ws > 1 and mode != "independent":
            eff = overlap_efficiency(agg["compute_ms"], agg["avg_ms"])
            rep.line(f"  - Scaling efficiency: {eff:.1f}% (compute / total time)")
    else:  # overlap
        rep.line(f"  - Average time per operation: {agg['avg_ms']:.3f} ms")
        actual = tflops_from(square_flops(n), agg["avg_ms"] / 1e3)
        extra["actual_tflops"] = actual
        rep.line(f"  - Actual TFLOPS: {actual:.2f} (FLOPs/Time)")
        rep.line(f"  - Compute-only TFLOPS: {agg['compute_only_tflops']:.2f} "
                 f"(GEMM alone, {agg['compute_ms']:.3f} ms)")
        if ws > 1:
            eff = overlap_efficiency(agg["compute_ms"], agg["avg_ms"])
            rep.line(f"  - Communication overhead: {100.0 - eff:.1f}% of each iteration is exposed comm")
            rep.line(f"  - Note: In data parallel, each GPU does full matrix multiply")
            rep.line(f"  - System is achieving {actual * ws:.2f} TFLOPS across {ws} GPUs")
        rep.line(f"  - Required FLOPs per operation: {square_flops(n) / 1e12:.2f} TFLOPs")

    # MI355X additions, identical for every kind.
    rep.line(f"  - Node TFLOPS (all FLOPs / slowest rank): {agg['node_tflops']:.2f}")
    ref1 = agg.get("single_gpu_tflops") or args.single_gpu_tflops
    if ref1:
        extra["single_gpu_tflops"] = ref1
        eff = scaling_efficiency(agg["node_tflops"], ws, ref1)
        extra["scaling_efficiency_vs_1gpu"] = eff
        rep.line(f"  - Scaling efficiency vs 1 GPU: {eff:.1f}%")
    if kind != "basic":
        pct = percent_of_peak(r.tflops if mode not in ("matrix_parallel", "ring_parallel")
                              else r.compute_only_tflops or 0.0,
                              peak, dtype)
        if pct is not None:
            extra["pct_peak"] = pct
    rep.line(f"  - Kernel: {r.kernel}")
    if agg.get("relerr") is not None:
        ok = agg["relerr"] < tolerance(dtype)
        extra["check_ok"] = ok
        rep.line(f"  - Check: max rel. error {agg['relerr']:.2e} ({'PASS' if ok else 'FAIL'})")
    return extra


def _completed(args, kind: str, mode: str, ctx: DistContext) -> set:
    """Sizes already recorded in ``--json`` for this (script, mode, dtype, ws, backend).

    Every rank reads the same file, so all ranks skip the same sizes."""
    import json
    import os

    if not args.json or not os.path.exists(args.json):
        return set()
    got = set()
    with open(args.json) as f:
        for line in f:
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if (r.get("script") == kind and r.get("mode") == mode and r.get("dtype") == args.dtype
                    and r.get("world_size") == ctx.world_size and r.get("backend") == args.backend
                    and bool(r.get("overlap", False)) == bool(args.overlap) and "error" not in r):
                got.add(int(r["n"]))
    return got


def dist_backend_name() -> str:
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return "none"
    be = dist.get_backend()
    return "RCCL" if be == "nccl" else be


def run_benchmarks(kind: str, ctx: DistContext, rep: Reporter, args) -> List[Dict]:
    k = KINDS[kind]
    mode = _mode_of(kind, args)
    dtype = dtype_from_name(args.dtype)
    rep.line(f"\n{'=' * k['width']}")
    rep.line(k["title"])
    rep.line("=" * k["width"])
    rep.line("Configuration:")
    if kind != "basic":
        rep.line(f"  - Mode: {mode}")
    rep.line(f"  - Number of GPUs: {ctx.world_size}" if ctx.is_cuda
             else f"  - Number of processes: {ctx.world_size}")
    rep.line(f"  - Data type: {dtype}")
    rep.line(f"  - Device: {'GPU (' + torch.cuda.get_device_name(ctx.device) + ')' if ctx.is_cuda else 'CPU'}")
    if not ctx.is_cuda:
        rep.line("  - GEMM: torch.matmul (CPU reference path)")
    elif args.backend == "native":
        rep.line("  - GEMM: native gfx950 MFMA kernels")
    else:
        rep.line("  - GEMM: torch.matmul (hipBLASLt), A/B comparison")
    if kind != "basic" and ctx.world_size > 1:
        coll = {"batch_parallel": f"all-reduce: {args.allreduce}",
                "matrix_parallel": f"all-gather: {args.allgather}",
                "model_parallel": f"all-gather: {args.allgather}",
                "ring_parallel": "ring P2P"}.get(mode, f"all-reduce: {args.allreduce}")
        rep.line(f"  - Collective: {coll} (backend {dist_backend_name()})")
    rep.line(f"  - Iterations per test: {args.iterations}")
    rep.line(f"  - Warmup iterations: {args.warmup}")
    hooks = testhooks.active()
    if hooks:  # negative-control fault injection: not a measurement
        rep.line(f"  - WARNING: test-only fault injection active ({', '.join(hooks)}): "
                 "collectives may race; timings are not measurements")
    rep.line(f"{'=' * k['width']}\n")
    out = []
    done = _completed(args, kind, mode, ctx) if getattr(args, "resume", False) else set()
    for n in args.sizes:
        if n <= 0:
            rep.line(f"\n  ERROR: invalid size {n}")
            continue
        if n in done:
            rep.line(f"\nSkipping {n}x{n}: already recorded in {args.json} (--resume)")
            continue
        bpe = bytes_per_element(dtype)
        rep.line(f"\nBenchmarking {n}x{n} matrix multiplication:")
        rep.line(f"  - Memory per matrix: {n * n * bpe / (1024 ** 3):.2f} GB ({dtype_name(dtype)})")
        if kind == "basic":
            obpe = bytes_per_element(_gemm_out_dtype(dtype))  # fp8 operands write a bf16 C
            rep.line(f"  - Total memory for A, B, C: {(2 * bpe + obpe) * n * n / (1024 ** 3):.2f} GB")
        else:
            rep.line(f"  - Mode: {mode}")
        if kind in ("distributed", "overlap"):
            rep.line("  - Running warmup and benchmark...")
        res, err, ref1 = None, None, None
        try:
            if getattr(args, "scaling_ref", False):
                ref1 = _single_gpu_reference(ctx, args, n, dtype)
            with marker(f"{kind}/{mode}/{n}x{n}/{dtype_name(dtype)}/ws{ctx.world_size}",
                        enabled=getattr(args, "profile", False) and ctx.is_cuda):
                res = run_mode(mode, _workload(args, n, dtype), ctx)
        except torch.cuda.OutOfMemoryError:
            err = f"Out of memory for {n}x{n} matrices"
        except Exception as e:  # reported by every rank, never swallowed
            err = f"{type(e).__name__}: {e}"
            if getattr(args, "debug", False):
                traceback.print_exc()
        if err is not None:
            print(f"[rank {ctx.rank}] ERROR: {err}", flush=True)
        if not all_ok(ctx, err is None):
            rep.line(f"\n  ERROR: {err or 'failed on another rank'}")
            out.append({"n": n, "mode": mode, "error": err or "failed on another rank"})
        else:
            agg = _aggregate(ctx, res)
            if ref1:
                agg["single_gpu_tflops"] = ref1
            extra = _print_results(kind, mode, rep, ctx, n, dtype, res, agg, args)
            rec = {"script": kind, "mode": mode, "n": n, "dtype": dtype_name(dtype),
                   "world_size": ctx.world_size, "device": ctx.device.type,
                   "backend": args.backend, "iterations": args.iterations,
                   "warmup": args.warmup, "tflops_rank0": res.tflops, "kernel": res.kernel,
                   "flops_per_iter_total": res.flops_total, **agg, **extra, **res.extra}
            if hooks:
                rec["test_hooks"] = hooks
            rep.record(rec)
            out.append(rec)
        del res
        if ctx.is_cuda:
            torch.cuda.empty_cache()
        barrier(ctx)
    return out


def main(kind: str, argv=None) -> int:
    parser = build_parser(kind)
    args = parser.parse_args(argv)
    if args.iterations < 1 or args.warmup < 0 or args.chunks < 0 or args.batch < 1:
        parser.error("--iterations must be >= 1, --batch >= 1, --warmup and --chunks >= 0")
    ctx = setup_distributed(args.device, timeout_s=args.timeout,
                            backend=None if args.dist_backend == "auto" else args.dist_backend)
    rep = Reporter(is_main=ctx.is_main, json_path=args.json)
    device_banner(rep, ctx.device)
    if ctx.is_main and ctx.is_cuda and (args.show_topology or
                                        (kind == "overlap" and torch.cuda.device_count() > 1)):
        from .utils.topology import topology_lines

        rep.line("\nGPU interconnect (xGMI on MI355X nodes):")
        for line in topology_lines():
            rep.line(f"  {line}")
    try:
        if ctx.world_size > 1 and kind != "basic" and not verify_collectives(ctx):
            rep.line("ERROR: Collective operations verification failed!")
            return 1
        run_benchmarks(kind, ctx, rep, args)
    finally:
        cleanup_distributed()
    w = KINDS[kind]["width"]
    rep.line(f"\n{'=' * w}")
    rep.line("Benchmark completed!")
    rep.line(f"{'=' * w}\n")
    return 0
