#!/usr/bin/env python3
"""Exactness screen of the thin-round W4S arms (PDMB_EXPERIMENTS=1 build):
x_fp8_w4s_thin / x_w4s_thin run the shipping W4S with the 256-tile round that
follows the grid's aspect (common.h thin_supertile: wide 4 x 64 / 8 x 32,
tall 64 x 4 / 32 x 8) instead of the 16 x 16 round. Only the tile order
changes, so each must be bitwise equal to the shipping W4S on random data,
and every tile must be written (the output starts as NaN). One JSON line per
case; exit 1 on failure.

    PDMB_EXPERIMENTS=1 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench
    python scripts/check_thin.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

CASES = [  # (M, N, K): wide 4 x 64 / 8 x 32 rounds, tall 64 x 4 / 32 x 8, square (unchanged order)
    (4096, 16384, 1024), (2048, 16384, 1024), (16384, 4096, 1024), (16384, 2048, 1024),
    (4096, 8192, 2048), (8192, 4096, 2048), (8192, 8192, 1024), (1024, 16384, 768),
]


def main():
    dev = torch.device("cuda", 0)
    bad = 0
    for dt, arm, base in ((torch.float8_e4m3fn, "x_fp8_w4s_thin", "fp8_w4s"),
                          (torch.bfloat16, "x_w4s_thin", "w4s")):
        for m, n, k in CASES:
            g = torch.Generator(device=dev).manual_seed(m + 3 * n + k)
            A = torch.randn(m, k, device=dev, generator=g).to(dt)
            if dt == torch.float8_e4m3fn:
                B = torch.randn(n, k, device=dev, generator=g).to(dt).t()  # column-major K x N
            else:
                B = torch.randn(k, n, device=dev, generator=g).to(dt)
            try:
                ref = gemm.matmul(A, B, kernel=base)
                outs = []
                for _ in range(2):
                    o = torch.full_like(ref, float("nan"))
                    gemm.matmul(A, B, out=o, kernel=arm)
                    outs.append(o)
            except (RuntimeError, ValueError) as e:
                print(json.dumps({"arm": arm, "shape": [m, n, k], "refused": str(e)[:80]}), flush=True)
                bad += 1
                continue
            same = all(bool(torch.equal(o, ref)) for o in outs)
            bad += not same
            print(json.dumps({"arm": arm, "shape": [m, n, k], "bitwise_eq": same}), flush=True)
    print(json.dumps({"failures": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
