#!/usr/bin/env python3
"""Run auto on a few wave-quantised shapes, once per tail setting, for a
rocprofv3 kernel trace of the tail plans' launches (profiles/r5n_tail_kernel_trace.md):

    rocprofv3 --kernel-trace --stats -d OUT -o tails -- python3 scripts/tail_trace.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

CASES = [("bfloat16", 6144, 6144, 6144), ("bfloat16", 6144, 4096, 4096),
         ("float8_e4m3fn", 6144, 6144, 6144), ("float32", 5120, 5120, 5120)]


def main() -> int:
    torch.manual_seed(0)
    for dname, m, n, k in CASES:
        dt = getattr(torch, dname)
        if dt == gemm.FP8:
            A, _ = gemm.fp8_quantize(torch.randn(m, k, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(k, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
        C = torch.empty(m, n, device="cuda", dtype=gemm.out_dtype(dt))
        for env in ("", "0"):  # auto's tail plan, then PDMB_TILE_TAIL=0 + PDMB_TAIL_REFINE=0 (no tail)
            for var in ("PDMB_TILE_TAIL", "PDMB_TAIL_REFINE"):
                if env:
                    os.environ[var] = env
                else:
                    os.environ.pop(var, None)
            for _ in range(10):
                gemm.matmul(A, B, out=C)
            torch.cuda.synchronize()
            print(dname, m, n, k, "tail" if not env else "no tail", gemm.tail_split_for(A, B, C), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
