#!/usr/bin/env python3
"""Exactness check of the bf16/fp16 W4 kernel (gemm_w4.hip) on the GPU:
small-integer operands make every fp32 partial sum exact, so C must equal the
fp64 product rounded once to the output dtype. Covers odd K-tile counts,
a batch, padded leading dimensions and both dtypes.

    python scripts/w4_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(1)
    ok = True
    for dt in (torch.bfloat16, torch.float16):
        for (b, M, N, K, pad) in [(1, 256, 256, 64, 0), (1, 512, 768, 128, 0), (1, 1024, 512, 192, 0),
                                  (1, 2304, 2048, 1024, 0), (3, 512, 512, 256, 0), (1, 768, 1280, 320, 64),
                                  (1, 4096, 4096, 4096, 0)]:
            Af = torch.randint(-3, 4, (b, M, K + pad), device="cuda", generator=g).to(dt)[..., :K]
            Bf = torch.randint(-3, 4, (b, K, N + pad), device="cuda", generator=g).to(dt)[..., :N]
            if b == 1:
                Af, Bf = Af[0], Bf[0]
            C = gemm.matmul(Af, Bf, kernel="w4")
            ref = (Af.double() @ Bf.double()).to(dt)
            e = torch.equal(C, ref)
            ok &= e
            print(dt, b, M, N, K, pad, "exact" if e else
                  f"MISMATCH maxdiff={(C.float() - ref.float()).abs().max().item()} "
                  f"bad={(C != ref).sum().item()}", flush=True)
    print("ALL OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
