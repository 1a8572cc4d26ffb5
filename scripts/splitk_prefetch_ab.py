#!/usr/bin/env python3
"""A/B of the S == 2 split-K reducer's row-ahead slot prefetch (splitk.h
``splitk_load_other``, GemmArgs::meet_prefetch) against the row-by-row
``splitk_row`` path, in ONE process: the switch is the environment variable
PDMB_SPLITK_PREFETCH (read per launch), flipped between interleaved arms.
Prints one JSON line per (shape, dtype, kernel): median TFLOPS per arm and
whether the two outputs are bitwise equal (they must be).

    python scripts/splitk_prefetch_ab.py [--rounds 7] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

CASES = [  # (dtype, M, N, K, kernel, S)
    ("bfloat16", 4096, 512, 4096, "t128", 2),
    ("bfloat16", 4096, 1024, 4096, "t128", 2),
    ("bfloat16", 2048, 2048, 2048, "t128", 2),
    ("bfloat16", 8192, 1024, 8192, "t256x128", 2),
    ("float8_e4m3fn", 4096, 512, 4096, "fp8_t128", 2),
    ("float8_e4m3fn", 8192, 1024, 8192, "fp8_t256x128", 2),
    ("float32", 4096, 512, 4096, "f32_t128", 2),
    ("float32", 4096, 1024, 4096, "f32_t128", 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    for dn, m, n, k, kern, S in CASES:
        dt = getattr(torch, dn)
        torch.manual_seed(0)
        if dt == gemm.FP8:
            A, _ = gemm.fp8_quantize(torch.randn(m, k, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(k, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
        C = torch.empty(m, n, device="cuda", dtype=gemm.out_dtype(dt))
        flops = 2.0 * m * n * k
        outs = {}
        for arm in ("1", "0"):
            os.environ["PDMB_SPLITK_PREFETCH"] = arm
            outs[arm] = gemm.matmul(A, B, kernel=kern, splitk=S).clone()
        torch.cuda.synchronize()
        same = bool(torch.equal(outs["1"], outs["0"]))
        res = {"1": [], "0": []}
        for r in range(a.rounds):
            for arm in (("1", "0") if r % 2 == 0 else ("0", "1")):
                os.environ["PDMB_SPLITK_PREFETCH"] = arm
                ms = gemm.bench_matmul(A, B, C, a.iters, 2, kernel=kern, splitk=S) / a.iters
                res[arm].append(flops / ms / 1e9)
        os.environ.pop("PDMB_SPLITK_PREFETCH", None)
        print(json.dumps({"dtype": dn, "m": m, "n": n, "k": k, "kernel": f"{kern}:{S}",
                          "prefetch_tflops": round(statistics.median(res["1"]), 1),
                          "rowwise_tflops": round(statistics.median(res["0"]), 1),
                          "gain": round(statistics.median(res["1"]) / statistics.median(res["0"]), 4),
                          "bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
