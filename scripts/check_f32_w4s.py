#!/usr/bin/env python3
"""Exactness screen of the streamed exact-fp32 W4 kernel (x_f32_w4s, experiment
build) against an fp64 reference and, bitwise, against its non-streamed form
(x_f32_w4_lean2: the same per-element accumulation order). Shapes cover one
and several tiles per workgroup, grids that are not multiples of the
workgroup count, batches, small-integer data (exact in fp32, so
any dropped, doubled or misplaced K-tile shows as a nonzero error) and a K the
kernel refuses (K / 32 odd, M or N edges). One JSON line per case; exit 1 on any failure.

    PDMB_EXPERIMENTS=1 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench
    python scripts/check_f32_w4s.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

CASES = [  # (batch, M, N, K, integer data): whole 256 x 256 tiles only (host-checked)
    (1, 256, 256, 128, True), (1, 4096, 4096, 256, True), (1, 8192, 8192, 512, False),
    (1, 5120, 3072, 1024, True), (1, 9216, 6912, 640, True), (3, 1024, 1024, 512, True),
    (1, 2304, 8960, 384, False), (1, 16384, 4096, 256, True), (1, 4352, 4608, 192, True),
]
REFUSED = [(512, 512, 96), (300, 512, 256), (512, 260, 256)]  # K / 32 odd; M, N edges


def main():
    dev = torch.device("cuda", 0)
    bad = 0
    for bt, m, n, k, exact in CASES:
        g = torch.Generator(device=dev).manual_seed(m * 7 + n + k)
        shp_a = (bt, m, k) if bt > 1 else (m, k)
        shp_b = (bt, k, n) if bt > 1 else (k, n)
        if exact:
            A = torch.randint(-3, 4, shp_a, device=dev, generator=g).float()
            B = torch.randint(-3, 4, shp_b, device=dev, generator=g).float()
        else:
            A = torch.randn(shp_a, device=dev, generator=g)
            B = torch.randn(shp_b, device=dev, generator=g)
        R = torch.matmul(A.double(), B.double())
        out = gemm.matmul(A, B, kernel="x_f32_w4s")
        ref = gemm.matmul(A, B, kernel="x_f32_w4_lean2")
        err = ((out.double() - R).norm() / R.norm().clamp_min(1e-30)).item()
        same = bool(torch.equal(out, ref))
        ok = (err == 0.0) if exact else (err < 1e-6)
        ok = ok and same and bool(torch.isfinite(out).all())
        bad += not ok
        print(json.dumps({"batch": bt, "m": m, "n": n, "k": k, "exact": exact, "relerr": err,
                          "bitwise_eq_lean2": same, "ok": ok}), flush=True)
    for m, n, k in REFUSED:
        A = torch.randn(m, k, device=dev)
        B = torch.randn(k, n, device=dev)
        try:
            gemm.matmul(A, B, kernel="x_f32_w4s")
            refused = False
        except RuntimeError:
            refused = True
        bad += not refused
        print(json.dumps({"m": m, "n": n, "k": k, "refused": refused, "ok": refused}), flush=True)
    print(json.dumps({"failures": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
