#!/usr/bin/env python3
"""Profiling driver: the native GEMM kernel(s) and torch.matmul (hipBLASLt) on the
same random operands, interleaved, a few launches each — run under
``rocprofv3 --kernel-trace`` or ``--pmc …`` to compare counters per kernel.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES ... --output-format csv -d out -- \
        python3 scripts/prof_gemm_arms.py --n 16384 --reps 4
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--kernels", default="auto", help="comma list of native kernels")
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    n = a.n
    torch.manual_seed(0)
    A = torch.randn(n, n, device="cuda", dtype=dt)
    B = torch.randn(n, n, device="cuda", dtype=dt)
    C = torch.empty(n, n, device="cuda", dtype=dt)
    ks = a.kernels.split(",")
    for _ in range(2):  # warm (clocks, caches, code objects)
        for k in ks:
            gemm.matmul(A, B, out=C, kernel=k)
        if not a.no_torch:
            torch.matmul(A, B, out=C)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        for k in ks:
            gemm.matmul(A, B, out=C, kernel=k)
        if not a.no_torch:
            torch.matmul(A, B, out=C)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
