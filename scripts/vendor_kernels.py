#!/usr/bin/env python3
"""Run the vendor library (hipBLASLt via torch.matmul / torch._scaled_mm) on given
shapes so a rocprofv3 kernel trace shows which kernel (macro tile, grid) it picks.

    rocprofv3 --kernel-trace --stats -d gpurun_out/vk -o vk -- python3 scripts/vendor_kernels.py \
        --dtype float8_e4m3fn --shapes 4096,4096,4096 8192,2048,8192
"""
import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--shapes", nargs="+", required=True, help="M,N,K")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    for s in a.shapes:
        m, n, k = (int(v) for v in s.split(","))
        if dt == torch.float8_e4m3fn:
            A = torch.randn(m, k, device="cuda").to(dt)
            B = torch.randn(n, k, device="cuda").to(dt).t()  # column-major
            one = torch.ones((), device="cuda")
            f = lambda: torch._scaled_mm(A, B, one, one, out_dtype=torch.bfloat16)  # noqa: E731
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
            f = lambda: torch.matmul(A, B)  # noqa: E731
        for _ in range(a.iters):
            f()
        torch.cuda.synchronize()
        print(f"{s} done", flush=True)


if __name__ == "__main__":
    main()
