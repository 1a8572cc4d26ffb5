#!/usr/bin/env python3
"""Single-GPU GEMM throughput: native gfx950 kernel vs torch.matmul (hipBLASLt).

Interleaves the arms in one process (cdna rule 24) on the same random data.
Usage: python scripts/gemm_perf.py --sizes 4096 8192 16384 --dtype bfloat16
       python scripts/gemm_perf.py --shapes 16384x2048x16384 8192x2048x16384   (MxNxK)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

DT = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
      "float8_e4m3fn": torch.float8_e4m3fn}


def scaled_mm_ms(A8, B8, out, iters, warmup):
    """hipBLASLt fp8 through torch._scaled_mm (None if this build lacks it)."""
    one = torch.ones((), device=A8.device)
    try:
        torch._scaled_mm(A8, B8, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    except Exception as e:  # noqa: BLE001
        print(f"# torch._scaled_mm unavailable: {e!r}"[:200], flush=True)
        return None
    f = lambda: torch._scaled_mm(A8, B8, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
    for _ in range(warmup):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


def torch_ms(A, B, out, iters, warmup):
    for _ in range(warmup):
        torch.matmul(A, B, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        torch.matmul(A, B, out=out)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[4096, 8192, 16384])
    ap.add_argument("--dtype", default="bfloat16", choices=list(DT))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--shapes", nargs="+", default=None,
                    help="rectangular MxNxK problems (e.g. the per-rank shards of matrix_parallel)")
    a = ap.parse_args()
    dt = DT[a.dtype]
    probs = ([tuple(int(x) for x in s.lower().split("x")) for s in a.shapes] if a.shapes
             else [(n, n, n) for n in a.sizes])
    for m, n, k in probs:
        torch.manual_seed(0)
        fp8 = dt == torch.float8_e4m3fn
        if fp8:  # per-tensor scaled e4m3, B column-major (alpha folds the scales)
            A, sa = gemm.fp8_quantize(torch.randn(m, k, device="cuda"))
            B, sb = gemm.fp8_quantize(torch.randn(k, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
        out = torch.empty(m, n, device="cuda", dtype=gemm.out_dtype(dt))
        flop = 2.0 * m * n * k
        res = {"n": n, "shape": f"{m}x{n}x{k}", "dtype": a.dtype,
               "kernel": gemm.kernel_for(A, B, out, kernel=a.kernel)}
        ours, ours_g, theirs = [], [], []
        for _ in range(a.rounds):
            ms = gemm.bench_matmul(A, B, out, a.iters, a.warmup, graph=False, kernel=a.kernel) / a.iters
            ours.append(flop / ms / 1e9)
            ms = gemm.bench_matmul(A, B, out, a.iters, a.warmup, graph=True, kernel=a.kernel) / a.iters
            ours_g.append(flop / ms / 1e9)
            if not a.no_torch:
                ms = (scaled_mm_ms(A, B, out, a.iters, a.warmup) if fp8
                      else torch_ms(A, B, out, a.iters, a.warmup))
                if ms is not None:
                    theirs.append(flop / (ms / a.iters) / 1e9)
        ref = torch.matmul(A.float(), B.float())
        C = gemm.matmul(A, B, kernel=a.kernel)
        res["relerr"] = ((C.float() - ref).norm() / ref.norm()).item()
        res["native_tflops"] = [round(x, 1) for x in ours]
        res["native_graph_tflops"] = [round(x, 1) for x in ours_g]
        if theirs:
            res["torch_tflops"] = [round(x, 1) for x in theirs]
        print(json.dumps(res), flush=True)
        del A, B, out, ref, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"# done in {time.time() - t0:.1f}s")
