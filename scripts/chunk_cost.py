#!/usr/bin/env python3
"""Compute-side cost of overlap chunking: one 16k bf16 GEMM issued as 1 / 2 / 4 /
8 / 16 row-chunk GEMMs (native W4 kernel), interleaved rounds, median TFLOPS.
Used to size the overlap chunk count (finer chunks shrink the exposed tail
collective; this measures what they cost the GEMM)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.partition import row_chunks  # noqa: E402


def main():
    n, iters, rounds = 16384, 10, 7
    torch.manual_seed(0)
    A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    C = torch.empty_like(A)
    variants = [1, 2, 4, 8, 16]
    res = {c: [] for c in variants}
    for _ in range(2 + rounds):
        for c in variants:
            rc = row_chunks(n, c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                for s, e in rc:
                    gemm.matmul(A[s:e], B, out=C[s:e])
            e1.record()
            e1.synchronize()
            res[c].append(2.0 * n ** 3 * iters / (e0.elapsed_time(e1) / 1e3) / 1e12)
    for c in variants:
        print(json.dumps({"n": n, "chunks": c, "median_tflops": round(statistics.median(res[c][2:]), 1),
                          "kernel": gemm.kernel_for(A[:n // c], B)}), flush=True)


if __name__ == "__main__":
    main()
