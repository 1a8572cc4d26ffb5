#!/usr/bin/env python3
"""Repeated-run race screen for the tile kernels (SURVEY §5 race detection):
each (kernel, shape) runs ``--reps`` times on exact small-integer operands (every
product and sum is exact in fp32, so every run must equal the float64 product
bit for bit); prints one JSON line per case with the number of bad runs and the
first bad element (row, column, got, want) if any.

    python scripts/race_screen.py [--reps 200] [--kernels f32_t128x2,f32_t128,t128x2]
    python scripts/race_screen.py --tails [--reps 50]   # auto's two-launch tail plans (bf16, fp8)
    python scripts/race_screen.py --splits [--reps 50]  # round 5: auto's 3- / 5- / 6-way splits, f32_t64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

SHAPES = [(256, 256, 32), (256, 256, 64), (256, 256, 96), (256, 256, 128), (512, 768, 192),
          (1024, 1024, 1024), (3072, 3072, 1024), (2304, 2304, 1024)]
# --tails: auto's wave-quantisation tail plans (a whole-wave launch, then a
# split-K launch whose slices meet in-kernel): the tile-range form on these
TAIL_SHAPES = [(6144, 6144, 6144), (6000, 6000, 6144), (7168, 7168, 7168), (5120, 5120, 5120), (4608, 4608, 3072),
               (6144, 4096, 4096), (3000, 7000, 5056)]
# exact fp32's tail (whole two-per-CU waves, then an f32_t128 split-K wave)
F32_TAIL_SHAPES = [(3072, 3072, 3072), (5120, 5120, 2048), (7168, 7168, 1024)]
# --splits (round 5): grids auto runs with a 3-way (bf16, fp32) or 5- / 6-way
# (fp32) split-K, and on the 64x128 fp32 tile
SPLIT_CASES = [("auto:bfloat16", (2560, 4096, 16384)), ("auto:bfloat16", (4608, 2048, 16384)),
               ("auto:bfloat16", (2560, 512, 8192)), ("auto:bfloat16", (3584, 2560, 16384)),
               ("auto:float32", (2560, 256, 8192)), ("auto:float32", (1536, 1536, 4096)),
               ("auto:float32", (1024, 256, 16384)), ("auto:float32", (512, 6400, 16384)),
               ("auto:float32", (4096, 512, 4096)), ("auto:float32", (2048, 512, 2048)),
               # round 5: split f32_t128x2 on < 2 tiles per CU, 8-way f32_t64
               ("auto:float32", (2560, 2048, 4096)), ("auto:float32", (3072, 1536, 2048)),
               ("auto:float32", (6144, 768, 16384)), ("auto:float32", (1000, 3000, 4096)),
               ("auto:float32", (768, 256, 16384)), ("auto:float32", (256, 768, 8192)),
               # round 5: small-grid split rules (T128 x 3 below 32 K-tiles per slice)
               ("auto:bfloat16", (768, 768, 4096)), ("auto:float16", (256, 768, 2048)),
               ("auto:bfloat16", (1024, 1024, 8192)), ("auto:float8_e4m3fn", (768, 768, 8192)),
               ("auto:float8_e4m3fn", (1000, 260, 8192)),
               # round 5: f32_t64x2 split on small fp32 grids
               ("auto:float32", (1536, 3072, 1024)), ("auto:float32", (1536, 1536, 4096)),
               ("auto:float32", (9216, 256, 16384)), ("auto:float32", (3584, 3584, 2048)),
               ("auto:float32", (4608, 4608, 4096))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--kernels", default="f32_t128x2,f32_t128,f32_256s,t128x2,t128")
    ap.add_argument("--tails", action="store_true",
                    help="screen auto's tail plans (bf16 and fp8, TAIL_SHAPES) instead")
    ap.add_argument("--splits", action="store_true",
                    help="screen auto's non-power-of-two split plans (SPLIT_CASES) instead")
    a = ap.parse_args()
    if a.splits:
        cases = SPLIT_CASES
    elif a.tails:
        cases = ([(kd, shp) for kd in ("auto:bfloat16", "auto:float8_e4m3fn") for shp in TAIL_SHAPES]
                 + [("auto:float32", shp) for shp in F32_TAIL_SHAPES])
    else:
        cases = [(kern, shp) for kern in a.kernels.split(",") for shp in SHAPES]
    for kern, (m, n, k) in cases:
        kern, _, dname = kern.partition(":")
        dt = getattr(torch, dname) if dname else (torch.float32 if kern.startswith("f32") else torch.bfloat16)
        fp8 = dt == gemm.FP8
        S = 0 if kern == "auto" else 1
        if True:
            g = torch.Generator(device="cuda").manual_seed(m + 3 * n + k)
            lo, hi = (-2, 3) if fp8 else (-3, 4)
            Af = torch.randint(lo, hi, (m, k), device="cuda", generator=g).float()
            Bf = torch.randint(lo, hi, (k, n), device="cuda", generator=g).float()
            if fp8:  # e4m3 operands (exact small integers), B column-major, bf16 C
                A, B = Af.to(dt), Bf.t().contiguous().to(dt).t()
            else:
                A, B = Af.to(dt), Bf.to(dt)
            want = torch.matmul(Af.double(), Bf.double())
            odt = gemm.out_dtype(dt)
            if odt != torch.float32:
                want = want.to(odt).double()  # the fp32-exact sum rounded once, as the kernel does
            C = torch.empty(m, n, device="cuda", dtype=odt)
            try:
                gemm.matmul(A, B, out=C, kernel=kern, splitk=S)
            except (RuntimeError, ValueError):
                continue  # the kernel does not take this shape (bf16 K % 64)
            bad, first = 0, None
            plan = list(gemm.tail_split_for(A, B, C)) if kern == "auto" else None
            split = {"kernel_run": gemm.kernel_for(A, B, C), "splitk": gemm.splitk_for(A, B, C)} \
                if kern == "auto" and a.splits else {}
            for _ in range(a.reps):
                C.fill_(float("nan"))
                gemm.matmul(A, B, out=C, kernel=kern, splitk=S)
                d = C.double() != want
                if bool(d.any()):
                    bad += 1
                    if first is None:
                        idx = d.nonzero()[0].tolist()
                        first = {"row": idx[0], "col": idx[1], "got": C[idx[0], idx[1]].item(),
                                 "want": want[idx[0], idx[1]].item(), "n_bad": int(d.sum().item())}
            torch.cuda.synchronize()
            print(json.dumps({"kernel": kern, "dtype": str(dt).replace("torch.", ""), "m": m, "n": n,
                              "k": k, "reps": a.reps, "bad_runs": bad, "first_bad": first,
                              **({"tail_split": plan} if plan else {}), **split}), flush=True)


if __name__ == "__main__":
    main()
