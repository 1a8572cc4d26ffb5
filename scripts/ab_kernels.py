#!/usr/bin/env python3
"""Interleaved A/B of native GEMM kernel variants in ONE process (cdna rule 24):
N rounds × K kernels on the same random operands; prints median/min TFLOPS per
kernel and checks every variant against the first one's output.

    python scripts/ab_kernels.py --kernels mfma256c,x_noprio --sizes 8192 16384 --rounds 5
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
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--sizes", type=int, nargs="+", default=[8192, 16384])
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ks = a.kernels.split(",")
    dt = getattr(torch, a.dtype)
    for n in a.sizes:
        torch.manual_seed(0)
        if dt == torch.float8_e4m3fn:  # e4m3 operands (scale 1), B column-major, bf16 C
            A, _ = gemm.fp8_quantize(torch.randn(n, n, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(n, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(n, n, device="cuda", dtype=dt)
            B = torch.randn(n, n, device="cuda", dtype=dt)
        C = torch.empty(n, n, device="cuda", dtype=gemm.out_dtype(dt))
        ref = gemm.matmul(A, B, kernel=ks[0])
        R = torch.matmul(A.float(), B.float())
        res = {k: [] for k in ks}
        errs = {}
        for k in ks:
            out = gemm.matmul(A, B, kernel=k)
            errs[k] = ((out.float() - R).norm() / R.norm()).item()  # diag_* builds are timing-only
        for _ in range(2):  # warm clocks
            for k in ks:
                gemm.bench_matmul(A, B, C, 5, 2, kernel=k)
        for _ in range(a.rounds):
            for k in ks:
                ms = gemm.bench_matmul(A, B, C, a.iters, 2, kernel=k) / a.iters
                res[k].append(2.0 * n ** 3 / ms / 1e9)
        for k in ks:
            print(json.dumps({"n": n, "kernel": k, "median_tflops": round(statistics.median(res[k]), 1),
                              "min": round(min(res[k]), 1), "max": round(max(res[k]), 1),
                              "relerr": errs[k]}), flush=True)
        del A, B, C, ref, R
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
