#!/usr/bin/env python3
"""One auto GEMM launch in a fresh process (the first launch of the kernel in
that process), exact-integer operands checked against fp64; one JSON line.
Run it many times, each under a short `timeout`, to screen the shipping
kernels for first-launch hangs (round 6: the streamed exact-fp32 experiment
hung there, profiles/r8rw_fp32_stream_hang.md).

    python scripts/cold_probe.py DTYPE M N K
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def main():
    dt = getattr(torch, sys.argv[1])
    m, n, k = (int(x) for x in sys.argv[2:5])
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    Af = torch.randint(-2, 3, (m, k), device=dev, generator=g).float()
    Bf = torch.randint(-2, 3, (k, n), device=dev, generator=g).float()
    if dt == gemm.FP8:
        A, B = Af.to(dt), Bf.t().contiguous().to(dt).t()
    else:
        A, B = Af.to(dt), Bf.to(dt)
    t0 = time.perf_counter()
    C = gemm.matmul(A, B)
    torch.cuda.synchronize()
    s = time.perf_counter() - t0
    want = torch.matmul(Af.double(), Bf.double()).to(gemm.out_dtype(dt)).double()
    print(json.dumps({"dtype": sys.argv[1], "m": m, "n": n, "k": k, "kernel": gemm.kernel_for(A, B),
                      "exact": bool(torch.equal(C.double(), want)), "s": round(s, 4)}), flush=True)


if __name__ == "__main__":
    main()
