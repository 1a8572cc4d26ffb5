#!/usr/bin/env python3
"""C-pitch probe: does the output's row pitch (ldc) change a GEMM's time?

The fp8 W4 tile timeline at one tile per CU (profiles/
r2_fp8_w4_tile_timeline_one_tile_per_cu.jsonl) has a 13.7 us epilogue at
8192 x 2048 x 8192 (4 KiB C rows) against 5.1 us at 4096^3 (8 KiB rows), for
the same 32 MiB of C. This times the auto kernel writing into C views of one
shape with different row pitches (ldc = N, N + pad, ...), interleaved in
rounds, next to the vendor library at ldc = N.

    python scripts/ldc_probe.py --dtype float8_e4m3fn --shapes 8192,2048,8192 4096,4096,4096
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["8192,2048,8192", "4096,4096,4096",
                                                    "2048,8192,8192"])
    ap.add_argument("--dtype", default="float8_e4m3fn")
    ap.add_argument("--pads", default="0,64,128,256,2048")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    pads = [int(p) for p in a.pads.split(",")]
    for s in a.shapes:
        m, n, k = (int(v) for v in s.split(","))
        torch.manual_seed(0)
        if dt == torch.float8_e4m3fn:
            A, _ = gemm.fp8_quantize(torch.randn(m, k, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(k, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
        odt = gemm.out_dtype(dt)
        outs = {p: torch.empty(m, n + p, device="cuda", dtype=odt)[:, :n] for p in pads}
        one = torch.ones((), device="cuda")
        ref = gemm.matmul(A, B, kernel=a.kernel)
        for p, C in outs.items():
            gemm.matmul(A, B, out=C, kernel=a.kernel)
            assert torch.equal(C, ref), p
        flops = 2.0 * m * n * k

        def vendor(out):
            if dt == torch.float8_e4m3fn:
                return torch._scaled_mm(A, B, one, one, out_dtype=torch.bfloat16, out=out)
            return torch.matmul(A, B, out=out)

        def t_vendor(iters):
            C = outs[0]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            vendor(C)
            e0.record()
            for _ in range(iters):
                vendor(C)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / iters

        arms = [f"pad{p}" for p in pads] + ["torch"]
        res = {x: [] for x in arms}

        def one_round(iters, keep):
            for p in pads:
                us = gemm.bench_matmul(A, B, outs[p], iters, 2, kernel=a.kernel) / iters * 1e3
                if keep:
                    res[f"pad{p}"].append(us)
            us = t_vendor(iters) * 1e3
            if keep:
                res["torch"].append(us)

        one_round(10, False)
        for _ in range(a.rounds):
            one_round(a.iters, True)
        for x in arms:
            med = statistics.median(res[x])
            print(json.dumps({"m": m, "n": n, "k": k, "dtype": a.dtype, "arm": x,
                              "kernel": a.kernel if x != "torch" else "vendor",
                              "median_us": round(med, 2), "tflops": round(flops / med / 1e6, 1),
                              "min_us": round(min(res[x]), 2)}), flush=True)
        del A, B, outs, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
