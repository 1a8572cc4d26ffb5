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
    ap.add_argument("--shape", default=None, help="M,N,K (instead of the square --n)")
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    n = a.n
    m, nn, kk = (int(x) for x in a.shape.split(",")) if a.shape else (n, n, n)
    torch.manual_seed(0)
    if dt == torch.float8_e4m3fn:  # per-tensor scaled e4m3, B column-major; torch arm = _scaled_mm
        A, _ = gemm.fp8_quantize(torch.randn(m, kk, device="cuda"))
        B, _ = gemm.fp8_quantize(torch.randn(kk, nn, device="cuda"), colmajor=True)
        one = torch.ones((), device="cuda")

        def torch_mm(A, B, out):
            torch._scaled_mm(A, B, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    else:
        A = torch.randn(m, kk, device="cuda", dtype=dt)
        B = torch.randn(kk, nn, device="cuda", dtype=dt)

        def torch_mm(A, B, out):
            torch.matmul(A, B, out=out)
    C = torch.empty(m, nn, device="cuda", dtype=gemm.out_dtype(dt))
    ks = a.kernels.split(",")
    for _ in range(2):  # warm (clocks, caches, code objects)
        for k in ks:
            gemm.matmul(A, B, out=C, kernel=k)
        if not a.no_torch:
            torch_mm(A, B, C)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        for k in ks:
            gemm.matmul(A, B, out=C, kernel=k)
        if not a.no_torch:
            torch_mm(A, B, C)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
