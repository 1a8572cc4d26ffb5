#!/usr/bin/env python3
"""Exactness screen of the lean W4S arm (x_w4s_lean, PDMB_EXPERIMENTS=1 build):
small-integer operands (every fp32 partial sum exact, one rounding to the
output dtype) against fp64, bitwise equal to the shipping W4S on random data
(the same per-element MFMA order), repeatable; bf16 and fp16; grids of 1-16
tiles per workgroup, every supertile mode (square, thin), batches, the
six-K-tile minimum and a long K. One JSON line per case; exit 1 on failure.

    PDMB_EXPERIMENTS=1 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench
    python scripts/check_w4s_lean.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

CASES = [  # (batch, M, N, K)
    (1, 4096, 4096, 384), (1, 8192, 8192, 1024), (1, 16384, 16384, 512), (1, 16384, 2048, 2048),
    (1, 2048, 16384, 1024), (2, 4096, 4096, 2048), (1, 8192, 4096, 8192), (1, 4096, 8192, 640),
    (1, 1024, 16384, 768), (3, 4096, 4096, 384),
]


def main():
    dev = torch.device("cuda", 0)
    bad = 0
    for dt in (torch.bfloat16, torch.float16):
        for bt, m, n, k in CASES:
            g = torch.Generator(device=dev).manual_seed(m + n + k + bt)
            sa, sb = ((bt, m, k), (bt, k, n)) if bt > 1 else ((m, k), (k, n))
            A = torch.randint(-3, 4, sa, device=dev, generator=g).to(dt)
            B = torch.randint(-3, 4, sb, device=dev, generator=g).to(dt)
            try:
                out = gemm.matmul(A, B, kernel="x_w4s_lean")
            except (RuntimeError, ValueError) as e:
                print(json.dumps({"dtype": str(dt), "shape": [bt, m, n, k], "refused": str(e)[:80]}), flush=True)
                bad += 1
                continue
            exact = bool(torch.equal(out, torch.matmul(A.double(), B.double()).to(dt)))
            Ar = torch.randn(sa, device=dev, generator=g).to(dt)
            Br = torch.randn(sb, device=dev, generator=g).to(dt)
            o1 = gemm.matmul(Ar, Br, kernel="x_w4s_lean")
            same = bool(torch.equal(o1, gemm.matmul(Ar, Br, kernel="w4s")))
            reps = all(torch.equal(gemm.matmul(Ar, Br, kernel="x_w4s_lean"), o1) for _ in range(3))
            ok = exact and same and reps
            bad += not ok
            print(json.dumps({"dtype": str(dt).replace("torch.", ""), "shape": [bt, m, n, k], "exact": exact,
                              "bitwise_eq_w4s": same, "repeatable": reps, "ok": ok}), flush=True)
    print(json.dumps({"failures": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
