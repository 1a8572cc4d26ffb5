#!/usr/bin/env python3
"""Repeated-run race screen for the tile kernels (SURVEY §5 race detection):
each (kernel, shape) runs ``--reps`` times on exact small-integer operands (every
product and sum is exact in fp32, so every run must equal the float64 product
bit for bit); prints one JSON line per case with the number of bad runs and the
first bad element (row, column, got, want) if any.

    python scripts/race_screen.py [--reps 200] [--kernels f32_t128x2,f32_t128,t128x2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

SHAPES = [(256, 256, 32), (256, 256, 64), (256, 256, 96), (256, 256, 128), (512, 768, 192),
          (1024, 1024, 1024)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--kernels", default="f32_t128x2,f32_t128,f32_256s,t128x2,t128")
    a = ap.parse_args()
    for kern in a.kernels.split(","):
        dt = torch.float32 if kern.startswith("f32") else torch.bfloat16
        for m, n, k in SHAPES:
            g = torch.Generator(device="cuda").manual_seed(m + 3 * n + k)
            A = torch.randint(-3, 4, (m, k), device="cuda", generator=g).to(dt)
            B = torch.randint(-3, 4, (k, n), device="cuda", generator=g).to(dt)
            want = torch.matmul(A.double(), B.double())
            if dt != torch.float32:
                want = want.to(dt).double()  # bf16 output: exact for these magnitudes (|C| <= 9 k)
            C = torch.empty(m, n, device="cuda", dtype=dt)
            try:
                gemm.matmul(A, B, out=C, kernel=kern, splitk=1)
            except (RuntimeError, ValueError):
                continue  # the kernel does not take this shape (bf16 K % 64)
            bad, first = 0, None
            for _ in range(a.reps):
                C.fill_(float("nan"))
                gemm.matmul(A, B, out=C, kernel=kern, splitk=1)
                d = C.double() != want
                if bool(d.any()):
                    bad += 1
                    if first is None:
                        idx = d.nonzero()[0].tolist()
                        first = {"row": idx[0], "col": idx[1], "got": C[idx[0], idx[1]].item(),
                                 "want": want[idx[0], idx[1]].item(), "n_bad": int(d.sum().item())}
            torch.cuda.synchronize()
            print(json.dumps({"kernel": kern, "m": m, "n": n, "k": k, "reps": a.reps, "bad_runs": bad,
                              "first_bad": first}), flush=True)


if __name__ == "__main__":
    main()
