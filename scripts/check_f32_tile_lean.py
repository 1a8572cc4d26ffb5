#!/usr/bin/env python3
"""Exactness screen of the lean exact-fp32 tile arms (x_f32_t128_lean,
x_f32_t128x2_lean, x_f32_t64_lean, x_f32_t64x2_lean; PDMB_EXPERIMENTS=1 build):
each against fp64 on small-integer data (exact in fp32) and, bitwise, against
its shipping kernel at the same split (the same per-element MFMA order). Shapes
cover M / N edge tiles, K / 32 odd (the clamped tail DMAs), batches, 2- to
8-way split-K and a long K (32-bit voffsets). One JSON line per case; exit 1 on
any failure.

    PDMB_EXPERIMENTS=1 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench
    python scripts/check_f32_tile_lean.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

ARMS = {"x_f32_t128_lean": "f32_t128", "x_f32_t128x2_lean": "f32_t128x2", "x_f32_t64_lean": "f32_t64",
        "x_f32_t64x2_lean": "f32_t64x2"}
CASES = [  # (batch, M, N, K, splitk)
    (1, 128, 128, 32, 1), (1, 1000, 1052, 320, 1), (1, 300, 200, 96, 1), (3, 384, 640, 256, 1),
    (1, 4096, 512, 4096, 1), (1, 4096, 1024, 4096, 2), (1, 1000, 1052, 4096, 3), (1, 700, 300, 8192, 8),
    (1, 2048, 2048, 2048, 1), (1, 129, 132, 1024, 1), (1, 512, 256, 65536, 4),
]


def main():
    dev = torch.device("cuda", 0)
    bad = 0
    for arm, base in ARMS.items():
        for bt, m, n, k, S in CASES:
            g = torch.Generator(device=dev).manual_seed(m * 7 + n + k + bt)
            shp_a = (bt, m, k) if bt > 1 else (m, k)
            shp_b = (bt, k, n) if bt > 1 else (k, n)
            A = torch.randint(-3, 4, shp_a, device=dev, generator=g).float()
            B = torch.randint(-3, 4, shp_b, device=dev, generator=g).float()
            R = torch.matmul(A.double(), B.double())
            try:
                ref = gemm.matmul(A, B, kernel=base, splitk=S)
                out = gemm.matmul(A, B, kernel=arm, splitk=S)
            except (RuntimeError, ValueError) as e:
                print(json.dumps({"arm": arm, "batch": bt, "m": m, "n": n, "k": k, "splitk": S,
                                  "refused": str(e)[:80]}), flush=True)
                continue
            reps = all(torch.equal(gemm.matmul(A, B, kernel=arm, splitk=S), out) for _ in range(3))
            exact = bool(torch.equal(out.double(), R))
            same = bool(torch.equal(out, ref))
            ok = exact and same and reps
            bad += not ok
            print(json.dumps({"arm": arm, "batch": bt, "m": m, "n": n, "k": k, "splitk": S, "exact": exact,
                              "bitwise_eq_base": same, "repeatable": reps, "ok": ok}), flush=True)
    print(json.dumps({"failures": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
